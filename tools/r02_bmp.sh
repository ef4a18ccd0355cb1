# probe: why bmp inflates slower than repeat (kernel split + lane/resolve phases)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/profb gpurun_out/phases_bmp.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/profb --output-format csv -- python3 tools/kernel_times.py 256 bmp,repeat 2 > gpurun_out/kt_bmp.txt 2>&1
cat gpurun_out/kt_bmp.txt | grep -v amdgpu.ids
find gpurun_out/profb -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | head -12
DMX_KINDS=bmp timeout -k 10 200 python tools/phases.py gpurun_out/phases_bmp.txt > /dev/null 2>&1
cat gpurun_out/phases_bmp.txt
