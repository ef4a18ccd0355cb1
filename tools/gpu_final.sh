# round-end refresh: bench (with sub-records), rocprof kernel stats of the bench command, phases
# (run after tools/profile_all.sh run + collect, so bench's traffic keys are current)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
head -c 600 gpurun_out/bench_final.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
find gpurun_out/prof -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | head -8
rm -f gpurun_out/phases.txt
DMX_KINDS=repeat,text timeout -k 10 200 python tools/phases.py gpurun_out/phases.txt > /dev/null 2>&1
cat gpurun_out/phases.txt
