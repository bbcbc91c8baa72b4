"""Per-dispatch reading of a rocprofv3 --pmc CSV directory: for every dispatch of the given
kernels, its duration (the CSV's timestamps), the clock GRBM_GUI_ACTIVE / 8 XCDs / duration
(MI355X_MICROARCH.md, DVFS give-back), and with SQ_INSTS_VALU the VALU issue per SIMD-cycle
(x 4 cycles per wave64 instruction / SIMDs in use / cycles).
usage: pmc_dispatch.py DIR [KERNEL_REGEX] [SIMDS_BY_DISPATCH_ORDER]"""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
simds = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else []
rows = collections.defaultdict(dict)
meta = {}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if not pat.search(k):
            continue
        key = (int(r["Dispatch_Id"]), k)
        rows[key][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[key] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size"]))
per_kernel = collections.Counter()
for (i, k), c in sorted(rows.items()):
    t0, t1, grid = meta[(i, k)]
    ms = (t1 - t0) / 1e6
    n = per_kernel[k]
    per_kernel[k] += 1
    out = {"dispatch": i, "kernel": k, "grid_threads": grid, "ms": round(ms, 3)}
    if "GRBM_GUI_ACTIVE" in c and ms > 0:
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        out["mhz"] = round(cyc / (ms * 1e-3) / 1e6, 1)
        s = simds[n] if n < len(simds) else 1024
        if "SQ_INSTS_VALU" in c:
            out["valu_issue_per_simd_cycle"] = round(c["SQ_INSTS_VALU"] * 4 / s / cyc, 3)
            out["simds"] = s
        if "SQ_LDS_IDX_ACTIVE" in c:
            out["lds_busy_frac"] = round(c["SQ_LDS_IDX_ACTIVE"] / (s / 4) / cyc, 3)
    for name in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "FETCH_SIZE"):
        if name in c:
            out[name] = int(c[name])
    print(out)
