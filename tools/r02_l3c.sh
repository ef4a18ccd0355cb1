# level 3 chain depth on the level-2 links: 16 (tree) vs 32 (ab/libdmx_d32.so)
set -e
echo "== depth 16"; timeout -k 10 300 python -u tools/kernel_times.py 256 text,mixed,bmp 3 2>&1 | grep -v amdgpu.ids
echo "== depth 32"; DMX_LIB=ab/libdmx_d32.so timeout -k 10 300 python -u tools/kernel_times.py 256 text,mixed,bmp 3 2>&1 | grep -v amdgpu.ids
