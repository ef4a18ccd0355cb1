# Quick per-kernel breakdown on the GPU box: rocprofv3 kernel stats of tools/kernel_times.py for
# each corpus:level in $SPECS (1 GiB, 3 deflate + 3 inflate calls), plus the DMX_PHASES timeline
# of repeat and text.  Results under gpurun_out/ks_*.  usage: SPECS="repeat:2 text:2" bash tools/gpu_kstats.sh
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SPECS=${SPECS:-"repeat:2 text:2"}
MIB=${MIB:-1024}
for spec in $SPECS; do
  c=${spec%%:*}; l=${spec#*:}
  rm -rf gpurun_out/ks_$c$l
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/ks_$c$l --output-format csv -- python3 tools/kernel_times.py $MIB $c $l > gpurun_out/ks_$c$l.txt 2>&1
  cat gpurun_out/ks_$c$l.txt | grep -v amdgpu.ids
  find gpurun_out/ks_$c$l -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | head -8
done
if [ "${PHASES:-1}" = 1 ]; then
  rm -f gpurun_out/phases.txt
  DMX_KINDS=${PH_KINDS:-repeat,text} timeout -k 10 200 python tools/phases.py gpurun_out/phases.txt > /dev/null 2>&1
  cat gpurun_out/phases.txt
fi
