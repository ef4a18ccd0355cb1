# block-parallel inflate bring-up: inflate parity tests, then timing of foreign streams
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "inflate" > gpurun_out/fb_tests.log 2>&1 || { tail -40 gpurun_out/fb_tests.log; exit 1; }
tail -3 gpurun_out/fb_tests.log
timeout -k 10 200 python -u tools/foreign_probe.py bmp:0:1 text:16:1 text:64:6 mixed:64:1 > gpurun_out/fb_probe.log 2>&1 || { cat gpurun_out/fb_probe.log; exit 1; }
cat gpurun_out/fb_probe.log
