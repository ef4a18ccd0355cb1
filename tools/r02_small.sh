# inflate at several sizes (lane count chosen by segment count), after the parity tests
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_containers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/small_tests.log 2>&1 || { tail -40 gpurun_out/small_tests.log; exit 1; }
tail -2 gpurun_out/small_tests.log
for mib in 64 256 512 1024; do
  echo "== $mib MiB"; timeout -k 10 200 python -u tools/kernel_times.py $mib repeat,text,mixed 2 2>&1 | grep -v amdgpu.ids
done
