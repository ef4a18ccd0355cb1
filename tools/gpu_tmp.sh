# scratch A/B script (developer aid; rewritten as needed)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in ${VARS:-u0 u1 u2}; do
  echo "== $v"
  DMX_LIB=ab/libdmx_$v.so timeout -k 10 200 python tools/kernel_times.py ${MIB:-256} ${KINDS:-text,repeat,bmp,mixed} ${LVL:-3} 2>&1 | grep -v "^W\|^E\|amdgpu.ids"
done
