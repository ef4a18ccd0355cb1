# ratio cost of the 9/6-bit code cap per corpus: the library built with 15/15-bit limits
# (ab/libdmx_cap15.so, tools/ab_build-style) against the tree's, level 2 and 3, 256 MiB
set -e
for lvl in 2 3; do
  echo "== cap 9/6, level $lvl"; timeout -k 10 300 python -u tools/kernel_times.py 256 repeat,text,mixed,zeros,random,bmp $lvl 2>&1 | grep -v amdgpu.ids
  echo "== cap 15/15, level $lvl"; DMX_LIB=ab/libdmx_cap15.so timeout -k 10 300 python -u tools/kernel_times.py 256 repeat,text,mixed,zeros,random,bmp $lvl 2>&1 | grep -v amdgpu.ids
done
