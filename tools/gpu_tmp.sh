# scratch A/B script (developer aid; rewritten as needed)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base sk; do
  echo "== $v"
  DMX_LIB=ab/libdmx_$v.so timeout -k 10 200 python tools/kernel_times.py 1024 repeat,text,mixed,zeros,bmp,random 2 2>&1 | grep -v "^W\|^E\|amdgpu.ids"
done
rm -f gpurun_out/ph_*.txt
for v in sk; do
  DMX_LIB=ab/libdmx_$v.so DMX_KINDS=repeat,text DMX_MIB=256 timeout -k 10 200 python tools/phases.py gpurun_out/ph_$v.txt > /dev/null 2>&1
  echo "== phases $v"; grep "^deflate\|^#" gpurun_out/ph_$v.txt
done
