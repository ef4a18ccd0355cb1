# Round-6 GPU check, part A: the changed tests first (path 5 truncation, serial bar, stream
# ordering of deflate_gather), then the whole GPU suite, then a HEAD kernel profile of the path-5
# fixed-code streams (the r05 CSV predates df05caf).  Results in gpurun_out/.
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ok_or_fail() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_path5_foreign.py tests/test_gpu_serial.py tests/test_gpu_multi.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r6a_changed.log 2>&1; rc=$?
grep -E "GPU |serial |truncated|PASSED|FAILED|XFAIL|XPASS|passed|failed" gpurun_out/r6a_changed.log | tail -40
ok_or_fail $rc || exit 1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_path5_foreign.py --ignore=tests/test_gpu_serial.py --ignore=tests/test_gpu_multi.py > gpurun_out/r6a_gpu_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r6a_gpu_tests.log | tail -12
ok_or_fail $rc || exit 1
rm -rf gpurun_out/r6_prof_foreign
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_prof_foreign --output-format csv -- python3 tools/foreign_probe.py single:mixed:16 zfixed:text:64 zfixed:mixed:32 > gpurun_out/r6_foreign.txt 2>&1
grep -E "path=" gpurun_out/r6_foreign.txt | tail -12
exit 0
