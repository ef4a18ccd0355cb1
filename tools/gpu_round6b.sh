# Round-6 GPU check, part B: config C4's 64 KiB blocks (parity at edge sizes, the 8 GiB run on
# the lane path), then the whole suite, then one bench line with the c4_64k sub-record.
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ok_or_fail() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_path5_foreign.py -v -s -x --timeout 300 --timeout-method thread > gpurun_out/r6b_p5.log 2>&1; rc=$?
grep -E "GPU |truncated|PASSED|FAILED|passed|failed" gpurun_out/r6b_p5.log | tail -30
[ $rc -eq 0 ] || exit 1
rm -rf gpurun_out/r6b_prof_foreign
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6b_prof_foreign --output-format csv -- python3 tools/foreign_probe.py single:mixed:16 zfixed:text:64 zfixed:mixed:32 > gpurun_out/r6b_foreign.txt 2>&1
grep -E "path=" gpurun_out/r6b_foreign.txt | tail -12
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "64KiB or roundtrip_oracle or compiled_reference" -v -s -x --timeout 300 --timeout-method thread > gpurun_out/r6b_64k.log 2>&1; rc=$?
grep -E "blocks|PASSED|FAILED|Error|error|passed|failed" gpurun_out/r6b_64k.log | tail -40
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_c4.py -v -s -x --timeout 500 --timeout-method thread > gpurun_out/r6b_c4.log 2>&1; rc=$?
grep -E "\[c4\]|PASSED|FAILED|passed|failed" gpurun_out/r6b_c4.log | tail -20
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/ -m gpu -q -x --timeout 300 --timeout-method thread --ignore=tests/test_gpu_c4.py > gpurun_out/r6b_gpu_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r6b_gpu_tests.log | tail -12
ok_or_fail $rc || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r6b_bench.json 2> gpurun_out/r6b_bench.err; rc=$?
python3 -c "import json;d=json.load(open('gpurun_out/r6b_bench.json'));print(d['value'],d['roofline']['frac'],d['roofline']['frac_inflate']);c=d['c4_64k'];m=d['corpora']['mixed'];print('c4_64k',c['ratio'],c['deflate_GBps'],c['inflate_GBps'],c['inflate_path'],c['kernel_ms']);print('mixed32',m['ratio'],m['deflate_GBps'],m['inflate_GBps'],m['kernel_ms'])"
exit $rc
