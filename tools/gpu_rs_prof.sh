# Developer aid: rocprof kernel stats + DMX_PHASES of the resolve for $LIBS (ab/libdmx_<name>.so,
# "base" = in-tree) on $KINDS at 1 GiB.  usage: gpurun -- 'bash tools/gpu_rs_prof.sh'
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in ${LIBS:-old base}; do
  lib=ab/libdmx_$v.so; [ $v = base ] && lib=deflate.hpp_amd/lib/libdmx.so
  for c in ${KINDS:-repeat zeros}; do
    rm -rf gpurun_out/rs_$v$c
    DMX_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/rs_$v$c --output-format csv -- python3 tools/kernel_times.py 1024 $c 2 > gpurun_out/rs_$v$c.txt 2>&1
    echo "== $v $c"; grep -v amdgpu.ids gpurun_out/rs_$v$c.txt
    python3 tools/kstat_brief.py $(find gpurun_out/rs_$v$c -name "*kernel_stats.csv") | head -8
  done
  rm -f gpurun_out/phases_$v.txt
  DMX_LIB=$lib DMX_MIB=1024 DMX_KINDS=$(echo ${KINDS:-repeat zeros} | tr ' ' ,) timeout -k 10 200 python tools/phases.py gpurun_out/phases_$v.txt > /dev/null 2>&1
  grep -A0 "inflate\|^#" gpurun_out/phases_$v.txt
done
