# round-end refresh: full GPU suite, bench (with sub-records), rocprof kernel stats, PMC HBM traffic, phases
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof gpurun_out/pmcF gpurun_out/pmcW
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
head -c 600 gpurun_out/bench_final.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
find gpurun_out/prof -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | head -8
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > gpurun_out/pmcF.json 2> gpurun_out/pmcF.err
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > gpurun_out/pmcW.json 2> gpurun_out/pmcW.err
for k in k_deflate_segments k_inflate_lanes k_inflate_resolve; do
  python tools/traffic.py gpurun_out/pmcF gpurun_out/pmcW repeat:1073741824:2:$k $k gpurun_out/traffic.json || true
done
rm -f gpurun_out/phases.txt
DMX_KINDS=repeat,text timeout -k 10 200 python tools/phases.py gpurun_out/phases.txt > /dev/null 2>&1
cat gpurun_out/phases.txt
