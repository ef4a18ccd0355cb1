set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_repeat.json 2> gpurun_out/bench_repeat.err
timeout -k 10 300 python bench.py --corpus text --no-cpu-baseline > gpurun_out/bench_text.json 2> gpurun_out/bench_text.err
