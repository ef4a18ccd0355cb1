set -e
mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "deflate_roundtrip or compiled_reference" > gpurun_out/fm.log 2>&1 || { tail -30 gpurun_out/fm.log; exit 1; }
tail -1 gpurun_out/fm.log
rm -f gpurun_out/ab.txt
for lib in ab/libdmx_l258.so deflate.hpp_amd/lib/libdmx.so ab/libdmx_l64.so ab/libdmx_l16.so; do
  echo "== $lib" >> gpurun_out/ab.txt
  DMX_LIB=$lib timeout -k 10 120 python tools/kernel_times.py 256 text,repeat,bmp,mixed 3 >> gpurun_out/ab.txt 2>&1
done
grep -v amdgpu.ids gpurun_out/ab.txt
