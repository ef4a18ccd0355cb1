# A/B on one box (developer aid): GPU tests of the working tree's build, then per-corpus kernel
# times of each ab/libdmx_<name>.so given in $LIBS ("base" = the in-tree build).
# usage: gpurun -- 'bash tools/gpu_ab.sh'   (MIB, KINDS, LEVEL, TESTS=0 to skip the tests)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    --ignore=tests/test_gpu_c4.py > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for r in 1 2; do
  for v in ${LIBS:-base skip}; do
    echo "== $v (pass $r)"
    lib=ab/libdmx_$v.so; [ $v = base ] && lib=deflate.hpp_amd/lib/libdmx.so
    DMX_LIB=$lib timeout -k 10 200 python tools/kernel_times.py ${MIB:-1024} ${KINDS:-repeat,text,mixed,bmp,zeros,random} ${LEVEL:-2} 2>&1 | grep -v "^W\|^E\|amdgpu.ids"
  done
done
