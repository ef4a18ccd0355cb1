set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof gpurun_out/pmcF gpurun_out/pmcW  # (also clear them locally before merging)
timeout -k 10 400 python bench.py > gpurun_out/bench_repeat.json 2> gpurun_out/bench_repeat.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcF --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcF.json 2> gpurun_out/pmcF.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcW --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcW.json 2> gpurun_out/pmcW.err
timeout -k 10 400 python bench.py --corpus text > gpurun_out/bench_text.json 2> gpurun_out/bench_text.err
