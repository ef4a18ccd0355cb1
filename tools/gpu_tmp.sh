set -e
mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "quirks or nonuniform or false_markers" > gpurun_out/q.log 2>&1 || { grep -v "^$" gpurun_out/q.log | tail -40; exit 1; }
grep -E "PASS|FAIL" gpurun_out/q.log
bash tools/gpu_check.sh
