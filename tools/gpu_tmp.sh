# scratch A/B script (developer aid; rewritten as needed)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    --ignore=tests/test_gpu_c4.py > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in 1 2; do for v in ${LIBS:-head tab}; do
  echo "== $v"
  DMX_LIB=ab/libdmx_$v.so timeout -k 10 200 python tools/kernel_times.py 1024 ${KINDS:-repeat,zeros,bmp,mixed,text} 2 2>&1 | grep -v "^W\|^E\|amdgpu.ids"
done; done
rm -f gpurun_out/ph_*.txt
for v in ${PHLIBS:-tab}; do
  DMX_LIB=ab/libdmx_$v.so DMX_KINDS=repeat DMX_MIB=256 timeout -k 10 200 python tools/phases.py gpurun_out/ph_$v.txt > /dev/null 2>&1
  echo "== phases $v"; grep "^inflate\|^#" gpurun_out/ph_$v.txt
done
