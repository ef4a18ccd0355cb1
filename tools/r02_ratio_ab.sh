# level-3 link rounds: parity tests, then L3 ratio/time variants on 256 MiB text + mixed
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "deflate" 2>&1 | tail -2
echo "== base"; timeout -k 10 200 python -u tools/kernel_times.py 256 text,mixed,repeat 3 2>&1 | grep -v amdgpu.ids
for n in r128 d32 r64d32; do
echo "== $n"; DMX_LIB=$PWD/build_ab/$n/libdmx.so timeout -k 10 200 python -u tools/kernel_times.py 256 text,mixed 3 2>&1 | grep -v amdgpu.ids
done
