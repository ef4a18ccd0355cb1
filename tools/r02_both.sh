# deflate + inflate check: GPU parity and container tests, kernel times, phases of both directions
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_containers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/both_tests.log 2>&1 || { tail -40 gpurun_out/both_tests.log; exit 1; }
tail -2 gpurun_out/both_tests.log
timeout -k 10 200 python -u tools/kernel_times.py 1024 repeat,text,mixed,zeros,random 2 > gpurun_out/kt_both.txt 2>&1
cat gpurun_out/kt_both.txt
rm -f gpurun_out/phases.txt
DMX_KINDS=repeat,text timeout -k 10 200 python tools/phases.py gpurun_out/phases.txt > /dev/null 2>&1
cat gpurun_out/phases.txt
