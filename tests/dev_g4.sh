set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof_r gpurun_out/prof_t
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r --output-format csv -- python3 tests/dev_time.py 1024 repeat > gpurun_out/pr.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_t --output-format csv -- python3 tests/dev_time.py 1024 text > gpurun_out/pt.txt 2>&1
