# deflate/inflate kernel times per corpus at S = 32 KiB and 16 KiB, levels 2 and 3
set -e
mkdir -p gpurun_out
for s in 32768 16384; do
for l in 2 3; do
DMX_SEG=$s timeout -k 10 200 python -u tools/kernel_times.py 1024 repeat,text,mixed,bmp,zeros,random $l > gpurun_out/kt_${s}_$l.txt 2>&1
echo "== S=$s L=$l"; cat gpurun_out/kt_${s}_$l.txt
done
done
