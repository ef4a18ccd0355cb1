set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in 16 8 32; do
  lib=deflate.hpp_amd/lib/libdmx_l$L.so; [ $L = 16 ] && lib=deflate.hpp_amd/lib/libdmx.so
  echo "# LN_LANES=$L" >> gpurun_out/lanes_ab.log
  DMX_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python -u tests/dev_time.py 1024 text,repeat >> gpurun_out/lanes_ab.log 2>&1
done
