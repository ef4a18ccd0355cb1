# last check of the round: GPU suite, bench with sub-records, smoke
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_last.log 2>&1 || { tail -40 gpurun_out/gpu_tests_last.log; exit 1; }
tail -1 gpurun_out/gpu_tests_last.log
timeout -k 10 400 python bench.py > gpurun_out/bench_last.json 2> gpurun_out/bench_last.err || { tail -20 gpurun_out/bench_last.err; exit 1; }
head -c 400 gpurun_out/bench_last.json; echo
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
