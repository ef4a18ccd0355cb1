# Round-6 evidence: every corpus's kernel stats + PMC traffic (tools/profile_all.sh run r06),
# then the bench line and a rocprof of the bench command.  Results under gpurun_out/.
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1500 bash tools/profile_all.sh run r06 > gpurun_out/prof_all.log 2>&1; rc=$?
tail -8 gpurun_out/prof_all.log
[ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/r6_bprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_bprof --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/r6_bench_prof.json 2> gpurun_out/r6_bench_prof.err; rc=$?
head -c 700 gpurun_out/r6_bench_prof.json; echo
exit $rc
