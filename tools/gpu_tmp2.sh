set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in text random repeat; do echo "== $k"; DMX_LIB=ab/libdmx_skdbg.so timeout -k 10 120 python tools/deflate_once.py $k 1 2 2>&1 | grep -v "^W\|amdgpu.ids" | head -40; done
