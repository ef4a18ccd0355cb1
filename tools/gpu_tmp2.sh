set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/skip_dbg.py 67108865 mixed 2>&1 | grep -v "^W\|amdgpu.ids"
LIBS="head early" PHLIBS="early" KINDS="repeat,zeros,bmp,mixed,text" bash tools/gpu_tmp.sh
rm -f gpurun_out/ph_*.txt
DMX_LIB=ab/libdmx_early.so DMX_KINDS=repeat DMX_MIB=256 timeout -k 10 200 python tools/phases.py gpurun_out/ph_b.txt > /dev/null 2>&1
grep "^deflate" gpurun_out/ph_b.txt
