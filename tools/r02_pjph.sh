# workgroup decoder (path 2) phase timeline on text and bmp (DMX_PHASES)
set -e
mkdir -p gpurun_out
rm -f gpurun_out/phases_pj.txt
DMX_INFLATE_PATH=2 DMX_KINDS=text,bmp,repeat timeout -k 10 200 python tools/phases.py gpurun_out/phases_pj.txt > /dev/null 2>&1
cat gpurun_out/phases_pj.txt
