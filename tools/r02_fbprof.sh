# path-5 kernel breakdown (rocprof stats) on zlib streams, after the deflate parity tests
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fb_tests.log 2>&1 || { tail -40 gpurun_out/fb_tests.log; exit 1; }
tail -2 gpurun_out/fb_tests.log
rm -rf gpurun_out/fbprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fbprof --output-format csv -- python3 tools/foreign_probe.py bmp:0:1 text:256:1 > gpurun_out/fbprof.log 2>&1
cat gpurun_out/fbprof.log | grep -v amdgpu.ids
find gpurun_out/fbprof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -30
