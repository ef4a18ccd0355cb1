# bench + rocprof kernel stats of the bench command (developer aid)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/bprof
timeout -k 10 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/bprof --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
find gpurun_out/bprof -name "*kernel_stats.csv" | head -1 | xargs head -8
