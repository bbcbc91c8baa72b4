"""Per-kernel summary of rocprofv3 --pmc CSV directories: each counter's mean per dispatch of
that kernel (the bench's warmup and timed launches alike; they do the same work)."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        print(f"== {d}")
        for (k, c), v in sorted(agg.items()):
            print(f"  {k:36s} {c:22s} {v / len(disp[k]):18.0f}  ({len(disp[k])} dispatches)")
