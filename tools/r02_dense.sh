# stored segments out of the heavy count: GPU suite, then mixed / random inflate times A/B
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_dense.log 2>&1 || { tail -40 gpurun_out/gpu_tests_dense.log; exit 1; }
tail -1 gpurun_out/gpu_tests_dense.log
for lib in base new; do
  L=""; [ $lib = base ] && L=ab/libdmx_base.so
  for mib in 256 512 1024; do
    echo "== $lib $mib"; DMX_LIB=$L timeout -k 10 200 python -u tools/kernel_times.py $mib mixed,random,repeat 2 2>&1 | grep -v amdgpu.ids
  done
done
