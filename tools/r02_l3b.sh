# level 3 on the level-2 candidate links vs the link rounds (ab/libdmx_base.so = HEAD), ratio and time
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "deflate" > gpurun_out/l3b_tests.log 2>&1 || { tail -40 gpurun_out/l3b_tests.log; exit 1; }
tail -2 gpurun_out/l3b_tests.log
echo "== base L3"; DMX_LIB=ab/libdmx_base.so timeout -k 10 300 python -u tools/kernel_times.py 256 repeat,text,mixed,zeros,random,bmp 3 2>&1 | grep -v amdgpu.ids
echo "== new L3"; timeout -k 10 300 python -u tools/kernel_times.py 256 repeat,text,mixed,zeros,random,bmp 3 2>&1 | grep -v amdgpu.ids
echo "== new L2"; timeout -k 10 300 python -u tools/kernel_times.py 256 repeat,text,bmp 2 2>&1 | grep -v amdgpu.ids
