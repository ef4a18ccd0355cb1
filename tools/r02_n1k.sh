# heavy route with 1024-lane workgroups (ranges >= 128 / 192 bits) against 512 lanes
set -e
for v in new n1k n1k192; do
  L=""; [ $v != new ] && L=ab/libdmx_$v.so
  for mib in 1 24 64; do
    echo "== $v $mib"; DMX_LIB=$L timeout -k 10 200 python -u tools/kernel_times.py $mib text,bmp,mixed 2 2>&1 | grep -v amdgpu.ids
  done
done
