# A/B of inflate kernel times (base library vs tree) + rocprof per-kernel stats of the tree
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
K=${AB_KINDS:-repeat,text,mixed}
for i in 1 2; do
  echo "== base $i"; DMX_LIB=ab/libdmx_base.so timeout -k 10 200 python -u tools/kernel_times.py 1024 $K 2 2>&1 | grep -v amdgpu.ids
  echo "== new $i"; timeout -k 10 200 python -u tools/kernel_times.py 1024 $K 2 2>&1 | grep -v amdgpu.ids
done
rm -rf gpurun_out/rsprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rsprof --output-format csv -- python3 tools/kernel_times.py 1024 $K 2 > /dev/null 2>&1
find gpurun_out/rsprof -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | grep -v "at::" | head -12
