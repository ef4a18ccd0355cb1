# heavy route at its limits: GPU suite, then inflate times 1..512 MiB (mode 6 by default)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_route.log 2>&1 || { tail -40 gpurun_out/gpu_tests_route.log; exit 1; }
tail -1 gpurun_out/gpu_tests_route.log
for mib in 1 24 64 128 256 512; do
  echo "== MiB $mib"; timeout -k 10 200 python -u tools/kernel_times.py $mib text,bmp,mixed,repeat 2 2>&1 | grep -v amdgpu.ids
done
