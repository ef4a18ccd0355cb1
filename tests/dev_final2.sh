set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/profT2
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/f2_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/f2_bench_repeat.json 2> gpurun_out/f2_bench_repeat.err
timeout -k 10 300 python bench.py --corpus text > gpurun_out/f2_bench_text.json 2> gpurun_out/f2_bench_text.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profT2 --output-format csv -- python3 bench.py --corpus text --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/f2_benchT_prof.json 2> gpurun_out/f2_benchT_prof.err
