# developer A/B: deflate stream hashes of lib/libdmx_old.so vs lib/libdmx.so, then phases + tests
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -f gpurun_out/ab_*.json gpurun_out/ph_ab.txt
DMX_LIB=$GRAFT_REPO_ROOT/deflate.hpp_amd/lib/libdmx_old.so timeout -k 10 200 python tests/dev_same.py gpurun_out/ab_old.json > gpurun_out/ab_old.log 2>&1
timeout -k 10 200 python tests/dev_same.py gpurun_out/ab_new.json > gpurun_out/ab_new.log 2>&1
cmp gpurun_out/ab_old.json gpurun_out/ab_new.json && echo "AB SAME" > gpurun_out/ab_result.txt || echo "AB DIFF" > gpurun_out/ab_result.txt
DMX_KINDS=repeat,text timeout -k 10 200 python tests/dev_phases.py gpurun_out/ph_ab.txt > /dev/null 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err
if [ -n "$DMX_TESTS" ]; then timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; fi
