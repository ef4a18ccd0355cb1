set -e
mkdir -p gpurun_out
rm -f gpurun_out/phases16.txt gpurun_out/phases32.txt
DMX_SEG=16384 DMX_KINDS=repeat,text timeout -k 10 200 python tools/phases.py gpurun_out/phases16.txt > /dev/null 2>&1
DMX_SEG=32768 DMX_KINDS=repeat,text timeout -k 10 200 python tools/phases.py gpurun_out/phases32.txt > /dev/null 2>&1
grep -v inflate gpurun_out/phases16.txt; grep -v inflate gpurun_out/phases32.txt
