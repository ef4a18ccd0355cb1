# scratch A/B script (developer aid; rewritten as needed)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -f gpurun_out/ph.txt; DMX_MIB=1024 DMX_KINDS=text timeout -k 10 200 python tools/phases.py gpurun_out/ph.txt 2>&1 | grep -v "^W\|^E" | grep -v "^deflate"
for v in 2048 0; do
  rm -rf gpurun_out/tmp_$v
  DMX_RWG_MIN=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tmp_$v --output-format csv -- python3 tools/kernel_times.py 1024 text 2 > /dev/null 2>&1
  python3 - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/tmp_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "inflate" in r['Name']:
        print(f"RWG={sys.argv[1]:5s} {r['Name'][:48]:48s} {r['Calls']:>4s} {float(r['AverageNs'])/1e3:10.1f} us")
PY
done
