# small streams: every segment over 256 B to the workgroup decoder (<= 1 candidate per CU)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_small2.log 2>&1 || { tail -40 gpurun_out/gpu_tests_small2.log; exit 1; }
tail -1 gpurun_out/gpu_tests_small2.log
for lib in base new; do
  L=""; [ $lib = base ] && L=ab/libdmx_base.so
  for mib in 1 4 8; do
    echo "== $lib $mib"; DMX_LIB=$L timeout -k 10 200 python -u tools/kernel_times.py $mib repeat,zeros,text,bmp,mixed,random 2 2>&1 | grep -v amdgpu.ids
  done
done
