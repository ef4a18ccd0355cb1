# device-side heavy route: GPU suite, then 1 GiB / 256 MiB inflate times against ab/libdmx_base.so
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_route2.log 2>&1 || { tail -40 gpurun_out/gpu_tests_route2.log; exit 1; }
tail -1 gpurun_out/gpu_tests_route2.log
for i in 1 2; do
for lib in base new; do
  L=""; [ $lib = base ] && L=ab/libdmx_base.so
  echo "== $lib 1 GiB"; DMX_LIB=$L timeout -k 10 200 python -u tools/kernel_times.py 1024 repeat,text,mixed,bmp,zeros,random 2 2>&1 | grep -v amdgpu.ids
done
done
