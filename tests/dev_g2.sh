set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
DMX_SEG=16384 timeout -k 10 200 python tests/dev_time.py 1024 repeat,text,zeros > gpurun_out/t16.txt 2>&1
rm -f gpurun_out/phases.txt
timeout -k 10 200 python tests/dev_phases.py > /dev/null 2>&1
