# Path-5 check on the GPU: the region probe (DMX_FB_DEBUG), then the third-party-stream file,
# then (unless quick) the whole GPU suite.  usage: bash tools/gpu_p5.sh [quick]
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/p5single.py 4 16 > gpurun_out/p5single.log 2>&1 || { tail -40 gpurun_out/p5single.log; exit 1; }
grep -E "^single|chain breaks|units:|repair|region" gpurun_out/p5single.log | head -40
timeout -k 10 600 python -u -m pytest tests/test_gpu_path5_foreign.py tests/test_gpu_serial.py -v -s --timeout 300 --timeout-method thread > gpurun_out/p5v.log 2>&1; rc=$?
grep -E "GPU |PASSED|FAILED|passed|failed|Error" gpurun_out/p5v.log | tail -24
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
if [ "$1" != quick ]; then
  timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_path5_foreign.py --ignore=tests/test_gpu_serial.py > gpurun_out/gpu_tests.log 2>&1; rc=$?
  grep -E "FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -12
  [ $rc -eq 0 ] || exit 1
fi
