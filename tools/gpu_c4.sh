# config C4 at full size (tests/test_gpu_c4.py), one test per process, each under its own limit
set -e
mkdir -p gpurun_out && cd $GRAFT_REPO_ROOT
for t in test_c4_full_8GiB_mixed_shards_one_gpu test_stream_over_4GiB_random; do
  DMX_DEBUG=1 DMX_RECS=1 timeout -k 10 240 python -u -m pytest tests/test_gpu_c4.py -m gpu -x -v -s --timeout 200 --timeout-method thread -k $t >> gpurun_out/c4.log 2>&1 || { tail -60 gpurun_out/c4.log; exit 1; }
done
tail -5 gpurun_out/c4.log
