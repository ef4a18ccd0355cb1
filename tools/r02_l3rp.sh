# level 3 match-round size A/B: 2048 (ab/libdmx_base.so), 256, 512 (tree), 1024
set -e
K="timeout -k 10 300 python -u tools/kernel_times.py 256 text,mixed,bmp,repeat 3"
echo "== rp 2048"; DMX_LIB=ab/libdmx_base.so $K 2>&1 | grep -v amdgpu.ids
echo "== rp 256"; DMX_LIB=ab/libdmx_rp256.so $K 2>&1 | grep -v amdgpu.ids
echo "== rp 512"; $K 2>&1 | grep -v amdgpu.ids
echo "== rp 1024"; DMX_LIB=ab/libdmx_rp1024.so $K 2>&1 | grep -v amdgpu.ids
echo "== tree level 2"; timeout -k 10 300 python -u tools/kernel_times.py 256 text,repeat 2 2>&1 | grep -v amdgpu.ids
