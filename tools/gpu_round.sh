# One GPU call for a development round: the GPU suite (path-5 foreign streams first), kernel
# stats + DMX_PHASES timelines, the foreign-stream probe with the reference's 1-core times.
# Everything lands under gpurun_out/.  usage: bash tools/gpu_round.sh [quick]
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_foreign.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/p5v.log 2>&1 || { tail -60 gpurun_out/p5v.log; exit 1; }
grep -E "GPU |passed|failed" gpurun_out/p5v.log | tail -12
if [ "$1" != quick ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/gpu_tests.log
fi
SPECS=${SPECS:-"repeat:2 text:2 random:2"} PH_KINDS=${PH_KINDS:-repeat,text} bash tools/gpu_kstats.sh > gpurun_out/kstats.log 2>&1 || { tail -30 gpurun_out/kstats.log; exit 1; }
grep -E "^(repeat|text|random|mixed|zeros|bmp) |k_deflate|k_inflate|^deflate|^# " gpurun_out/kstats.log | cut -c1-400
if [ -n "$AB" ]; then  # A/B of ab/libdmx_<name>.so builds against the in-tree one
  LIBS="base $AB" TESTS=0 MIB=1024 KINDS=${AB_KINDS:-repeat,text,mixed,bmp} bash tools/gpu_ab.sh > gpurun_out/ab.log 2>&1 || { tail -30 gpurun_out/ab.log; exit 1; }
  cat gpurun_out/ab.log
fi
if [ -n "$AB3" ]; then  # the same at level 3 (256 MiB)
  LIBS="base $AB3" TESTS=0 MIB=256 LEVEL=3 KINDS=${AB3_KINDS:-text,mixed,repeat} bash tools/gpu_ab.sh > gpurun_out/ab3.log 2>&1 || { tail -30 gpurun_out/ab3.log; exit 1; }
  cat gpurun_out/ab3.log
fi
