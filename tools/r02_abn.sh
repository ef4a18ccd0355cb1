# A/B of several builds on one box: AB_LIBS="base s1 tree" (tree = the working tree's library)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
K=${AB_KINDS:-repeat,text,mixed}
MB=${AB_MB:-1024}
for i in 1 2; do
  for L in ${AB_LIBS:-base tree}; do
    if [ "$L" = tree ]; then lib=""; else lib=ab/libdmx_$L.so; fi
    echo "== $L $i"; DMX_LIB=$lib timeout -k 10 200 python -u tools/kernel_times.py $MB $K 2 2>&1 | grep -v amdgpu.ids
  done
done
