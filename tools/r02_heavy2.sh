# heavy routing: the new test, then small streams with every candidate on the workgroup decoder
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "heavy or c3 or golden" 2>&1 | tail -3
for mib in 1 8 96; do
  for h in 2048 1; do
    echo "== MiB $mib heavy $h"; DMX_HEAVY_BYTES=$h timeout -k 10 200 python -u tools/kernel_times.py $mib bmp,text,repeat,zeros 2 2>&1 | grep -v amdgpu.ids
  done
done
