set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/prof gpurun_out/ph_base.txt
DMX_KINDS=repeat,text timeout -k 10 200 python tests/dev_phases.py gpurun_out/ph_base.txt > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
