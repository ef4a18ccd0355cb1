# path-5 virtual units: the foreign-stream tests, then the whole GPU suite
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_foreign.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/p5v.log 2>&1 || { tail -60 gpurun_out/p5v.log; exit 1; }
grep -E "GPU|PASS|FAIL" gpurun_out/p5v.log | tail -20
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
