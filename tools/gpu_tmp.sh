# scratch A/B script (developer aid; rewritten as needed)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tmp_tests.log 2>&1 || { tail -30 gpurun_out/tmp_tests.log; exit 1; }
tail -1 gpurun_out/tmp_tests.log
for v in 1 2 4 8; do
  echo "== DMX_LN_PIECES=$v"
  DMX_LN_PIECES=$v timeout -k 10 200 python tools/kernel_times.py 1024 ${KINDS:-repeat,text,mixed,bmp,zeros} 2 2>&1 | grep -v "^W\|^E\|amdgpu.ids"
done
