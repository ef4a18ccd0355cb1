# Round-6 GPU check, part C: 64 KiB segments with 16-lane waves and split-half resolve.
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "64KiB or roundtrip_oracle or compiled_reference or nonuniform" -q -x --timeout 300 --timeout-method thread > gpurun_out/r6c_64k.log 2>&1; rc=$?
tail -3 gpurun_out/r6c_64k.log
[ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/r6c_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c_prof --output-format csv -- python3 tools/c4_probe.py mixed 1024 > gpurun_out/r6c_probe.txt 2>&1; rc=$?
cat gpurun_out/r6c_probe.txt | grep seg=
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py -q -s -x --timeout 500 --timeout-method thread > gpurun_out/r6c_c4.log 2>&1; rc=$?
grep -E "\[c4\]|passed|failed" gpurun_out/r6c_c4.log | tail -12
exit $rc
