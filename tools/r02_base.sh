# round-2 baseline: GPU suite sanity, deflate/inflate phases, foreign-stream (serial path) timing
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python -u tools/foreign_probe.py bmp:0:1 text:16:1 > gpurun_out/foreign.log 2>&1
cat gpurun_out/foreign.log
rm -f gpurun_out/phases.txt
DMX_KINDS=repeat,text timeout -k 10 200 python tools/phases.py gpurun_out/phases.txt > /dev/null 2>&1
cat gpurun_out/phases.txt
DMX_SEG=16384 timeout -k 10 200 python -u tools/kernel_times.py 1024 repeat,text > gpurun_out/t16.txt 2>&1
cat gpurun_out/t16.txt
