"""Developer aid (not a test): HBM traffic per launch from two rocprofv3 --pmc passes.

argv: fetch_dir write_dir key kernel_substring [traffic.json]; env DMX_ROUND: the round tag recorded
with the entry (bench.py reports only entries of its own round)
FETCH_SIZE and WRITE_SIZE are in KB per dispatch; on gfx950 FETCH_SIZE counts half the bytes of
wide streaming reads (MI355X_MICROARCH.md, HBM section), so it is doubled.  The per-launch
average over the dispatches whose kernel name contains kernel_substring is stored under key."""
import csv
import glob
import json
import os
import sys


def newest(root, pattern):
    """The newest run's file under root (gpurun merges each box's results into the local
    gpurun_out/, so older runs' files can sit beside it: they describe other kernels)."""
    files = glob.glob(os.path.join(root, "**", pattern), recursive=True)
    return [max(files, key=os.path.getmtime)] if files else []


def per_dispatch(root, counter, sub):
    vals = {}
    for f in newest(root, "*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter or sub not in row.get("Kernel_Name", ""):
                    continue
                k = (f, row.get("Dispatch_Id", row.get("Correlation_Id", "")))
                vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


fetch_dir, write_dir, key, sub = sys.argv[1:5]
out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), "profiles", "traffic.json")
fv = per_dispatch(fetch_dir, "FETCH_SIZE", sub)
wv = per_dispatch(write_dir, "WRITE_SIZE", sub)
if not fv or not wv:
    sys.exit(f"no dispatches of {sub}: fetch {len(fv)} write {len(wv)}")
fetch = 2 * 1024 * sum(fv) / len(fv)
write = 1024 * sum(wv) / len(wv)
tj = json.load(open(out)) if os.path.exists(out) else {}
tj[key] = round(fetch + write)
tj[key + ":detail"] = {"fetch_bytes_x2": round(fetch), "write_bytes": round(write),
                       "dispatches": [len(fv), len(wv)], "round": os.environ.get("DMX_ROUND", "")}
json.dump(tj, open(out, "w"), indent=1, sort_keys=True)
print(key, tj[key], tj[key + ":detail"])
