# Round-6 GPU check, part F: region map fast path -- path-5 tests (all shapes), kernel profile.
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_path5_foreign.py -v -s -x --timeout 300 --timeout-method thread > gpurun_out/r6f_p5.log 2>&1; rc=$?
grep -E "GPU |truncated|FAILED|passed|failed" gpurun_out/r6f_p5.log | tail -14
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -k "path5 or foreign or quirks or c3" --timeout 300 --timeout-method thread > gpurun_out/r6f_par.log 2>&1; rc=$?
tail -2 gpurun_out/r6f_par.log
[ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/r6f_prof_foreign
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6f_prof_foreign --output-format csv -- python3 tools/foreign_probe.py single:mixed:16 zfixed:text:64 zfixed:mixed:32 > gpurun_out/r6f_foreign.txt 2>&1
grep -E "path=" gpurun_out/r6f_foreign.txt | tail -12
python3 tools/kstat_brief.py gpurun_out/r6f_prof_foreign/runc/*_kernel_stats.csv | head -8
exit 0
