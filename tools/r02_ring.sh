# path-5 unit decode through an LDS ring: GPU suite, then foreign-stream inflate times A/B
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ring.log 2>&1 || { tail -40 gpurun_out/gpu_tests_ring.log; exit 1; }
tail -1 gpurun_out/gpu_tests_ring.log
for lib in base new; do
  L=""; [ $lib = base ] && L=ab/libdmx_base.so
  echo "== $lib"; DMX_LIB=$L timeout -k 10 300 python -u tools/foreign_probe.py bmp:0:1 text:64:1 mixed:64:6 2>&1 | grep -v amdgpu.ids
done
