# heavy-candidate routing (mode 6): GPU suite, then kernel times with it off / at 2 KiB / 4 KiB
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_heavy.log 2>&1 || { tail -40 gpurun_out/gpu_tests_heavy.log; exit 1; }
tail -2 gpurun_out/gpu_tests_heavy.log
for mib in 1 24 64; do
  for h in 0 2048 4096; do
    echo "== MiB $mib heavy $h"; DMX_HEAVY_BYTES=$h timeout -k 10 200 python -u tools/kernel_times.py $mib bmp,text,mixed,repeat 2 2>&1 | grep -v amdgpu.ids
  done
done
