set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/fbprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/fbprof --output-format csv -- python3 tools/foreign_probe.py bmp:0:1 text:64:6 > gpurun_out/fbprof.log 2>&1
cat gpurun_out/fbprof.log
find gpurun_out/fbprof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -30
