"""Summarize rocprofv3 --pmc CSV directories: per-dispatch average of each counter."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        rows = list(csv.DictReader(open(f)))
        agg = collections.defaultdict(float)
        disp = set()
        for r in rows:
            agg[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
        print(f"== {d} ({len(disp)} dispatches)")
        for k, v in sorted(agg.items()):
            print(f"  {k[0]:40s} {k[1]:24s} {v / len(disp):16.0f}")
