"""Developer aid: short per-kernel table (calls, average us) of rocprofv3 kernel_stats.csv files."""
import csv
import sys

for f in sys.argv[1:]:
    for row in csv.DictReader(open(f)):
        name = row["Name"].split("(")[0].replace("void ", "").replace("dmx::", "")
        print(f"  {name[:44]:44s} {int(row['Calls']):4d} {float(row['AverageNs']) / 1e3:9.1f} us")
