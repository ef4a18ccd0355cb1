set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/profT gpurun_out/pmcTF gpurun_out/pmcTW
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profT --output-format csv -- python3 bench.py --corpus text --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/benchT_prof.json 2> gpurun_out/benchT_prof.err
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcTF --output-format csv -- python3 bench.py --corpus text --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcTF.json 2> gpurun_out/pmcTF.err
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcTW --output-format csv -- python3 bench.py --corpus text --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmcTW.json 2> gpurun_out/pmcTW.err
