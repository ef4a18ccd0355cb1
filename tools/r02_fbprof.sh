# path 5 kernel split on the C3 stream (zlib-1 of the 25 MB bmp stand-in) and 64 MiB text zlib-1
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/proffb
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/proffb --output-format csv -- python3 tools/foreign_probe.py bmp:0:1 > gpurun_out/fb_probe.txt 2>&1
grep -v "^W20\|^E20\|amdgpu.ids" gpurun_out/fb_probe.txt | tail -5
find gpurun_out/proffb -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | head -14
