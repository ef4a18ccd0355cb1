# probe: the workgroup decoder (path 2) against the lane decoder (path 4) per corpus
set -e
mkdir -p gpurun_out
for p in 4 2; do
  echo "== path $p"; DMX_INFLATE_PATH=$p timeout -k 10 200 python -u tools/kernel_times.py 256 bmp,text,repeat,mixed 2 2>&1 | grep -v amdgpu.ids
done
