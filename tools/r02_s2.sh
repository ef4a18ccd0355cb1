# round-2 session-2 checkpoint: full GPU suite, foreign-stream timing, bench (repeat + text), kernel stats
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u tools/foreign_probe.py bmp:0:1 text:64:1 text:64:6 mixed:64:1 > gpurun_out/foreign.log 2>&1
cat gpurun_out/foreign.log
timeout -k 10 300 python bench.py > gpurun_out/bench_repeat.json 2> gpurun_out/bench_repeat.err
cat gpurun_out/bench_repeat.json
timeout -k 10 300 python bench.py --corpus text --no-cpu-baseline > gpurun_out/bench_text.json 2> gpurun_out/bench_text.err
cat gpurun_out/bench_text.json
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
find gpurun_out/prof -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-8
