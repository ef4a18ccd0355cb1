# Path-5 A/B on one box (developer aid): rocprof kernel stats of tools/foreign_probe.py, one
# stream spec at a time, for the in-tree build ("base") and each ab/libdmx_<name>.so in $LIBS.
# usage: gpurun -- 'LIBS="base scan4k" bash tools/gpu_ab_p5.sh'   (SPECS: foreign_probe specs)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/abp5
for spec in ${SPECS:-bmp:0:1 text:64:1}; do
  for v in ${LIBS:-base}; do
    lib=ab/libdmx_$v.so; [ $v = base ] && lib=deflate.hpp_amd/lib/libdmx.so
    d=gpurun_out/abp5/$v/${spec//:/_}; mkdir -p gpurun_out/abp5/$v
    DMX_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d --output-format csv -- \
      python3 tools/foreign_probe.py $spec > $d.txt 2>&1 || { tail -20 $d.txt; exit 1; }
    echo "== $v $spec $(grep 'path=' $d.txt | tail -1 | cut -c1-160)"
    cut -d, -f1-4 $(find $d -name "*kernel_stats.csv") | grep "k_fb" | sed 's/(.*)"//' | cut -c1-100
  done
done
# pdecode / k_fb_units phase cycles (DMX_FB_DEBUG) of each build
for spec in ${SPECS:-bmp:0:1 text:64:1}; do
  for v in ${LIBS:-base}; do
    lib=ab/libdmx_$v.so; [ $v = base ] && lib=deflate.hpp_amd/lib/libdmx.so
    f=gpurun_out/abp5/dbg_${v}_${spec//:/_}.txt
    DMX_LIB=$lib DMX_FB_DEBUG=1 timeout -k 10 120 python3 tools/foreign_probe.py $spec > $f 2>&1 || true
    echo "== debug $v $spec"; grep "pdecode cycles\|pdecode header\|k_fb_units cycles\|k_fb_check\|host us\|longest" $f | tail -6 | cut -c1-300
  done
done
