# workgroup decoder range length: path-2 times at 256 MiB and the heavy route at 24 MiB / 1 GiB bmp
set -e
for v in new m192 m384; do
  L=""; [ $v != new ] && L=ab/libdmx_$v.so
  echo "== $v path 2"; DMX_LIB=$L DMX_INFLATE_PATH=2 timeout -k 10 200 python -u tools/kernel_times.py 256 text,mixed 2 2>&1 | grep -v amdgpu.ids
  echo "== $v route"; DMX_LIB=$L timeout -k 10 200 python -u tools/kernel_times.py 24 text,bmp 2 2>&1 | grep -v amdgpu.ids
done
