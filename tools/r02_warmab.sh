# PJ_WARM variants: path-2 inflate times (256 MiB) per warm-up length
set -e
for v in w128 new w320 w512; do
  L=""; [ $v != new ] && L=ab/libdmx_$v.so
  echo "== $v"; DMX_LIB=$L DMX_INFLATE_PATH=2 timeout -k 10 200 python -u tools/kernel_times.py 256 text,bmp,mixed 2 2>&1 | grep -v amdgpu.ids
done
