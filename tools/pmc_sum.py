"""Developer aid (not a test): per-kernel sums and per-dispatch averages of the counters in a
rocprofv3 --pmc output directory.  argv: dir [kernel_substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if sub not in k:
            continue
        name = k.split("(")[0][-40:]
        acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[name].add((f, row.get("Dispatch_Id", "")))
for name, cs in acc.items():
    nd = max(1, len(disp[name]))
    print(name, f"dispatches={nd}")
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {v / nd:16.1f} per dispatch")
