# Round-6 GPU check, part G: repair units inside regions on exact chunk entries; whole suite.
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ok_or_fail() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_path5_foreign.py tests/test_gpu_foreign_1GiB.py -v -s -x --timeout 300 --timeout-method thread > gpurun_out/r6g_p5.log 2>&1; rc=$?
grep -E "GPU |truncated|FAILED|passed|failed" gpurun_out/r6g_p5.log | tail -14
[ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/r6g_prof_foreign
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6g_prof_foreign --output-format csv -- python3 tools/foreign_probe.py single:mixed:16 zfixed:text:64 zfixed:mixed:32 > gpurun_out/r6g_foreign.txt 2>&1
grep -E "path=" gpurun_out/r6g_foreign.txt | tail -12
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_c4.py --ignore=tests/test_gpu_path5_foreign.py --ignore=tests/test_gpu_foreign_1GiB.py > gpurun_out/r6g_gpu_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r6g_gpu_tests.log | tail -12
ok_or_fail $rc
