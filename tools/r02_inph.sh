# inflate phase timelines (lanes slots 0-4, resolve 5-7) on repeat and text
set -e
mkdir -p gpurun_out
rm -f gpurun_out/phases.txt
DMX_KINDS=repeat,text,mixed timeout -k 10 200 python tools/phases.py gpurun_out/phases.txt > /dev/null 2>&1
grep -v "^deflate" gpurun_out/phases.txt
