set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in 16 8 24; do
  lib=deflate.hpp_amd/lib/libdmx_r$L.so; [ $L = 16 ] && lib=deflate.hpp_amd/lib/libdmx.so
  echo "# LN_RING_LOW=$L" >> gpurun_out/ring_ab.log
  DMX_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python -u tests/dev_time.py 1024 text,repeat >> gpurun_out/ring_ab.log 2>&1
done
timeout -k 10 300 python bench.py --corpus text --no-cpu-baseline > gpurun_out/bench_text_d2d.json 2> gpurun_out/bench_text_d2d.err
