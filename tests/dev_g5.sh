set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
rm -rf gpurun_out/prof_r gpurun_out/prof_t
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r --output-format csv -- python3 tests/dev_time.py 1024 repeat,zeros,random > gpurun_out/pr.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_t --output-format csv -- python3 tests/dev_time.py 1024 text > gpurun_out/pt.txt 2>&1
