# Round-6 refresh after the resolve change: the whole GPU suite (C4 included), then the
# per-corpus profiles + PMC traffic, then the full bench line.
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r6i_tests.log 2>&1 || { tail -30 gpurun_out/r6i_tests.log; exit 1; }
tail -2 gpurun_out/r6i_tests.log
timeout -k 10 1500 bash tools/profile_all.sh run r06 > gpurun_out/prof_all.log 2>&1
tail -3 gpurun_out/prof_all.log
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 1; }
head -c 400 gpurun_out/bench_final.json; echo
rm -rf gpurun_out/r6_bprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_bprof --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/r6_bench_prof.json 2> gpurun_out/r6_bench_prof.err
