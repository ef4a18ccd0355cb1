# deflate check: GPU parity tests, 1 GiB kernel times at S = 32 KiB and 16 KiB, phases
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_containers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/df2_tests.log 2>&1 || { tail -40 gpurun_out/df2_tests.log; exit 1; }
tail -2 gpurun_out/df2_tests.log
timeout -k 10 200 python -u tools/kernel_times.py 1024 repeat,text,mixed,zeros,random 2 > gpurun_out/kt_df2.txt 2>&1
cat gpurun_out/kt_df2.txt
DMX_SEG=16384 timeout -k 10 200 python -u tools/kernel_times.py 1024 repeat,text 2 > gpurun_out/kt_df2_16.txt 2>&1
echo "S=16K"; cat gpurun_out/kt_df2_16.txt
rm -f gpurun_out/phases.txt
DMX_KINDS=repeat,text timeout -k 10 200 python tools/phases.py gpurun_out/phases.txt > /dev/null 2>&1
grep -v inflate gpurun_out/phases.txt
