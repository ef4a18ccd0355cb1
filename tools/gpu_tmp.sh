# scratch A/B script (developer aid; rewritten as needed)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DMX_LIB=ab/libdmx_sk.so timeout -k 10 120 python tools/skip_dbg.py 67108865 mixed 2>&1 | grep -v "^W\|amdgpu.ids"
DMX_LIB=ab/libdmx_sk.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    --ignore=tests/test_gpu_c4.py > gpurun_out/ab_tests_sk.log 2>&1 || { tail -30 gpurun_out/ab_tests_sk.log; exit 1; }
tail -1 gpurun_out/ab_tests_sk.log
for r in 1 2; do for v in base sk; do
  echo "== $v"
  DMX_LIB=ab/libdmx_$v.so timeout -k 10 200 python tools/kernel_times.py 1024 repeat,text,mixed,zeros,bmp,random 2 2>&1 | grep -v "^W\|^E\|amdgpu.ids"
done; done
