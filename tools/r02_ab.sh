# A/B on one box: kernel times of ab/libdmx_base.so against the working tree's library, alternated
set -e
mkdir -p gpurun_out
K=${AB_KINDS:-repeat,text,mixed}
for i in 1 2; do
  echo "== base $i"; DMX_LIB=ab/libdmx_base.so timeout -k 10 200 python -u tools/kernel_times.py 1024 $K 2 2>&1 | grep -v amdgpu.ids
  echo "== new $i"; timeout -k 10 200 python -u tools/kernel_times.py 1024 $K 2 2>&1 | grep -v amdgpu.ids
done
