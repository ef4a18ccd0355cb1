# full GPU suite + bench without extras + kernel stats
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-extras > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
cat gpurun_out/bench_quick.json
find gpurun_out/prof -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | head -16
