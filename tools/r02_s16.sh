set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "deflate_roundtrip" 2>&1 | tail -1
DMX_SEG=16384 timeout -k 10 200 python -u tools/kernel_times.py 1024 repeat,text,mixed,zeros,random 2 2>&1 | grep -v amdgpu.ids
