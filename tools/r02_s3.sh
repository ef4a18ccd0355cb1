# new bench (sub-records) + kernel times at S = 32/16 KiB, levels 2/3
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
for s in 16384 32768; do
for l in 2 3; do
DMX_SEG=$s timeout -k 10 200 python -u tools/kernel_times.py 1024 repeat,text,mixed,zeros,random $l > gpurun_out/kt_${s}_$l.txt 2>&1
echo "== S=$s L=$l"; cat gpurun_out/kt_${s}_$l.txt
done
done
