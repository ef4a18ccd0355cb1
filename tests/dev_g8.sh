set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -f gpurun_out/ph_*.txt
for fl in 0 1 2 4; do DMX_DF_FLAGS=$fl timeout -k 10 100 python tests/dev_phases.py gpurun_out/ph_$fl.txt > /dev/null 2>&1; done
