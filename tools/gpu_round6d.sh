# Round-6 GPU check, part D: DMX_PHASES of the 64 KiB lane decoder against 32 KiB (why 4x), and
# the path-5 fixed-code region map with the arithmetic code (tests + kernel profile).
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -f gpurun_out/r6d_phases.txt
DMX_PHASES=$GRAFT_REPO_ROOT/gpurun_out/r6d_phases.txt timeout -k 10 300 python3 tools/c4_probe.py mixed 256 > gpurun_out/r6d_probe.txt 2>&1; rc=$?
cat gpurun_out/r6d_probe.txt | grep seg=
grep inflate gpurun_out/r6d_phases.txt | awk '{print substr($0,1,400)}' | sort | uniq -c | sort -rn | head -6
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_path5_foreign.py -v -s -x --timeout 300 --timeout-method thread > gpurun_out/r6d_p5.log 2>&1; rc=$?
grep -E "GPU |truncated|FAILED|passed|failed" gpurun_out/r6d_p5.log | tail -14
[ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/r6d_prof_foreign
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6d_prof_foreign --output-format csv -- python3 tools/foreign_probe.py single:mixed:16 zfixed:text:64 zfixed:mixed:32 > gpurun_out/r6d_foreign.txt 2>&1
grep -E "path=" gpurun_out/r6d_foreign.txt | tail -12
exit 0
