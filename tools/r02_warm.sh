# workgroup decoder warm-up: GPU suite, pj phases, A/B against ab/libdmx_base.so
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_warm.log 2>&1 || { tail -40 gpurun_out/gpu_tests_warm.log; exit 1; }
tail -1 gpurun_out/gpu_tests_warm.log
rm -f gpurun_out/phases_pj2.txt
DMX_INFLATE_PATH=2 DMX_KINDS=text,bmp timeout -k 10 200 python tools/phases.py gpurun_out/phases_pj2.txt > /dev/null 2>&1
grep -v deflate gpurun_out/phases_pj2.txt
for lib in base new; do
  L=""; [ $lib = base ] && L=ab/libdmx_base.so
  for mib in 1 24 64; do
    echo "== $lib MiB $mib"; DMX_LIB=$L timeout -k 10 200 python -u tools/kernel_times.py $mib text,bmp,mixed 2 2>&1 | grep -v amdgpu.ids
  done
  echo "== $lib path 2 256 MiB"; DMX_LIB=$L DMX_INFLATE_PATH=2 timeout -k 10 200 python -u tools/kernel_times.py 256 text,bmp,repeat 2 2>&1 | grep -v amdgpu.ids
done
