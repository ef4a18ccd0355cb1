set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base new base new; do
  lib=deflate.hpp_amd/lib/libdmx_$v.so; [ $v = new ] && lib=deflate.hpp_amd/lib/libdmx.so
  echo "# $v" >> gpurun_out/lut_ab.log
  DMX_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python -u tests/dev_time.py 1024 text,repeat >> gpurun_out/lut_ab.log 2>&1
done
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/lut_gpu_tests.log 2>&1
