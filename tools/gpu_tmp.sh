# round-3 working script: correctness of the new paths, then an A/B of deflate kernel times
set -e
mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "false_markers or segment_starts or deflate_roundtrip or compiled_reference or 256MiB" > gpurun_out/fm.log 2>&1 || { tail -30 gpurun_out/fm.log; exit 1; }
tail -2 gpurun_out/fm.log
for lib in ab/libdmx_base.so ab/libdmx_nosplit.so deflate.hpp_amd/lib/libdmx.so ab/libdmx_base.so deflate.hpp_amd/lib/libdmx.so; do
  echo "== $lib" >> gpurun_out/ab.txt
  DMX_LIB=$lib timeout -k 10 120 python tools/kernel_times.py 256 repeat,text,mixed >> gpurun_out/ab.txt 2>&1
done
cat gpurun_out/ab.txt
bash tools/gpu_c4.sh
