"""Developer aid (not a test): sum rocprofv3 counter_collection.csv rows per kernel and counter.

argv: directory searched recursively for *counter_collection.csv; optional kernel-name filter."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "")
            if filt and filt not in k:
                continue
            tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
print(json.dumps({k: dict(v) for k, v in tot.items()}, indent=1, sort_keys=True))
