"""Per-launch counters from a rocprofv3 --pmc run (FETCH_SIZE SQ_INSTS_VALU) -> JSON for bench.py.

FETCH_SIZE is reported in KiB per dispatch; on gfx950 it counts exactly half of the bytes of
16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM section), so bytes = 2 * 1024 * KiB.
SQ_INSTS_VALU is the device-wide count of wave64 VALU instructions per dispatch.
usage: python tools/traffic.py <pmc_dir> <out.json>"""
import collections
import csv
import glob
import json
import sys

agg = collections.defaultdict(list)
for f in glob.glob(f"{sys.argv[1]}/*counter_collection.csv"):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        c = r["Counter_Name"]
        if c not in ("FETCH_SIZE", "SQ_INSTS_VALU"):
            continue
        per[(r["Dispatch_Id"], c)] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0].replace("void ", "")
    for (d, c), v in per.items():
        agg[names[d] + ("" if c == "FETCH_SIZE" else "_valu")].append(v)
out = {k: int((1 if k.endswith("_valu") else 2 * 1024) * sum(v) / len(v)) for k, v in agg.items()}
out["_note"] = ("<kernel>: FETCH_SIZE KiB x 1024 x 2 (gfx950 half-count correction); "
                "<kernel>_valu: SQ_INSTS_VALU; means per dispatch")
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(out)
