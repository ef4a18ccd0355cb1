# path-5 checks + timings (developer script): tests, probe, rocprof kernel stats of C3 and more
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "${SEL:-path5 or foreign or c3 or quirk or zlib}" > gpurun_out/t5.log 2>&1 || { tail -30 gpurun_out/t5.log; exit 1; }
tail -2 gpurun_out/t5.log
DMX_FB_DEBUG=${FBDBG:-} timeout -k 10 200 python tools/foreign_probe.py ${SPECS:-bmp:0:1 text:256:1 text:1024:1 mixed:256:6} > gpurun_out/fp.log 2>&1
grep -v "^W\|^E" gpurun_out/fp.log
rm -rf gpurun_out/p5prof
for sp in ${PROF:-bmp:0:1 mixed:256:6}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p5prof/$sp --output-format csv -- python3 tools/foreign_probe.py $sp > /dev/null 2>&1
  python3 - "$sp" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/p5prof/{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{sys.argv[1]:14s} {r['Name'][:40]:40s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:10.1f} us")
PY
done
