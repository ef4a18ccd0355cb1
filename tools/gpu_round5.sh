# Round-5 GPU evidence, part 1: the whole GPU suite (third-party streams and the serial decoder
# first), then rocprofv3 kernel stats of the path-5 fixed-code streams and of the serial decoder.
# Results under gpurun_out/; usage: bash tools/gpu_round5.sh
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ok_or_fail() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_path5_foreign.py tests/test_gpu_serial.py -v -s --timeout 300 --timeout-method thread > gpurun_out/p5v.log 2>&1; rc=$?
grep -E "GPU |serial |PASSED|FAILED|passed|failed" gpurun_out/p5v.log | grep -v print | tail -24
ok_or_fail $rc || exit 1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_path5_foreign.py --ignore=tests/test_gpu_serial.py > gpurun_out/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -12
ok_or_fail $rc || exit 1
rm -rf gpurun_out/prof_foreign gpurun_out/prof_serial
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_foreign --output-format csv -- python3 tools/foreign_probe.py single:mixed:16 zfixed:text:64 zfixed:mixed:32 bmp:0:1 > gpurun_out/foreign.txt 2>&1
grep -E "path=" gpurun_out/foreign.txt | tail -12
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial --output-format csv -- python3 tools/serial_probe.py 16 > gpurun_out/serial_probe16.txt 2>&1
grep -E "MB/s" gpurun_out/serial_probe16.txt
exit 0
