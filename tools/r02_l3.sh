# level-3 chains: GPU parity tests, kernel times at L2 and L3
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/l3_tests.log 2>&1 || { tail -40 gpurun_out/l3_tests.log; exit 1; }
tail -2 gpurun_out/l3_tests.log
timeout -k 10 300 python -u tools/kernel_times.py 1024 text,mixed,repeat,zeros 3 > gpurun_out/kt_l3.txt 2>&1
cat gpurun_out/kt_l3.txt
timeout -k 10 200 python -u tools/kernel_times.py 1024 text,repeat 2 > gpurun_out/kt_l2.txt 2>&1
cat gpurun_out/kt_l2.txt
