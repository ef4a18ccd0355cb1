set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 90 python -u tests/dev_time.py 256 mixed,random,bmp,repeat,text > gpurun_out/fp_kinds.log 2>&1
DMX_SEG=16384 timeout -k 10 90 python -u tests/dev_time.py 256 mixed,random,bmp,text 3 > gpurun_out/fp_kinds16.log 2>&1
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/fp_gpu_tests.log 2>&1
