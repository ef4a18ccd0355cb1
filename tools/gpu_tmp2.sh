set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -f gpurun_out/ph_*.txt
DMX_LIB=ab/libdmx_phdbg.so DMX_KINDS=repeat DMX_MIB=256 timeout -k 10 200 python tools/phases.py gpurun_out/ph_dbg.txt > /dev/null 2>&1
grep "^deflate\|^#" gpurun_out/ph_dbg.txt
