set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 200 python tests/dev_time.py 1024 repeat,zeros,random,text > gpurun_out/t.txt 2>&1
rm -f gpurun_out/phases.txt; timeout -k 10 200 python tests/dev_phases.py > /dev/null 2>&1
