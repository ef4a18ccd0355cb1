set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/final_gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/final_bench_repeat.json 2> gpurun_out/final_bench_repeat.err
timeout -k 10 300 python bench.py --corpus text > gpurun_out/final_bench_text.json 2> gpurun_out/final_bench_text.err
