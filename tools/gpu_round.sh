# One GPU call for a development round: the GPU suite (path-5 foreign streams first), kernel
# stats + DMX_PHASES timelines, the foreign-stream probe with the reference's 1-core times.
# Everything lands under gpurun_out/.  usage: bash tools/gpu_round.sh [quick]
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
# a test that fails (exit 1) does not stop the run; a crash, abort or time limit does
ok_or_fail() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [ -n "$P5PROBE" ]; then
  timeout -k 10 300 python -u tools/p5single.py $P5PROBE > gpurun_out/p5single.log 2>&1; rc=$?
  grep -E "^single|chain breaks|units:|repair" gpurun_out/p5single.log | head -60
  ok_or_fail $rc || exit 1
fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_path5_foreign.py -v -s --timeout 300 --timeout-method thread > gpurun_out/p5v.log 2>&1; rc=$?
grep -E "GPU |PASSED|FAILED|passed|failed|Error" gpurun_out/p5v.log | tail -16
ok_or_fail $rc || exit 1
if [ "$1" != quick ]; then
  timeout -k 10 900 python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread --ignore=tests/test_gpu_path5_foreign.py > gpurun_out/gpu_tests.log 2>&1; rc=$?
  grep -E "FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -12
  ok_or_fail $rc || exit 1
fi
SPECS=${SPECS:-"repeat:2 text:2 random:2"} PH_KINDS=${PH_KINDS:-repeat,text} bash tools/gpu_kstats.sh > gpurun_out/kstats.log 2>&1 || { tail -30 gpurun_out/kstats.log; exit 1; }
grep -E "^(repeat|text|random|mixed|zeros|bmp) |k_deflate|k_inflate|^deflate|^# " gpurun_out/kstats.log | cut -c1-400
if [ -n "$AB" ]; then  # A/B of ab/libdmx_<name>.so builds against the in-tree one
  LIBS="base $(ls ab 2>/dev/null | sed -n "s/^libdmx_\(.*\)\.so$/\1/p" | tr "\n" " ")" TESTS=0 MIB=1024 KINDS=${AB_KINDS:-repeat,text,mixed,bmp} bash tools/gpu_ab.sh > gpurun_out/ab.log 2>&1 || { tail -30 gpurun_out/ab.log; exit 1; }
  cat gpurun_out/ab.log
fi
if [ -n "$AB3" ]; then  # the same at level 3 (256 MiB)
  LIBS="base $AB3 $([ -f ab/libdmx_both.so ] && echo both)" TESTS=0 MIB=256 LEVEL=3 KINDS=${AB3_KINDS:-text,mixed,repeat} bash tools/gpu_ab.sh > gpurun_out/ab3.log 2>&1 || { tail -30 gpurun_out/ab3.log; exit 1; }
  cat gpurun_out/ab3.log
fi
