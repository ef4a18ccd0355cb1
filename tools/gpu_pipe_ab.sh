# Developer aid: deflate chunk pipeline A/B (DMX_DF_PIPE values) on one box, 1 GiB level 2.
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for p in ${PIPES:-0 8 4 16}; do
    echo "== pipe $p (pass $r)"
    DMX_DF_PIPE=$p timeout -k 10 200 python tools/kernel_times.py ${MIB:-1024} ${KINDS:-repeat,text,mixed,zeros,random,bmp} ${LEVEL:-2} 2>&1 | grep -v "^W\|^E\|amdgpu.ids"
  done
done
