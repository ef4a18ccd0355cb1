set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in 1 2 3; do for v in head out8; do echo "== $v"; DMX_LIB=ab/libdmx_$v.so timeout -k 10 200 python tools/kernel_times.py 1024 repeat,zeros,text 2 2>&1 | grep -v "^W\|^E\|amdgpu.ids"; done; done
