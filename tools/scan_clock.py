"""What holds the candidate scan's clock: the default workload (1024 x 4 MiB, resident) scanned
with the scan's workgroups capped at 256 (all CUs) down to 32 (PFSCDC_SCAN_GRID).  A clock held
down by chip power rises as fewer CUs work; a per-CU limit (LDS, issue) would not move it.
Prints one JSON line per cap: median scan / hash ms, in-kernel spans and clocks."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pfs_amd import _lib  # noqa: E402
from pfs_amd.cdc import ChunkParams, Chunker  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
files = int(sys.argv[2]) if len(sys.argv) > 2 else 1024  # 32768: the bench's 128 GiB step
grids = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 192, 128, 96, 64, 32, 0]
fbytes = 4 << 20
offs = np.arange(files + 1, dtype=np.uint64) * np.uint64(fbytes)
c = Chunker(ChunkParams(), 0)
data = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
c.fill_synthetic(data, offs, 0xC2)
digest = None
for grid in grids:
    _lib.set_knob("PFSCDC_SCAN_GRID", grid)
    rows = []
    for _ in range(reps + 1):
        r = c.scan(data, offs)
        rows.append(c.timings())
    rows = rows[1:]
    d = r.segments.tobytes().__hash__()
    digest = digest if digest is not None else d
    med = {k: round(statistics.median(x[k] for x in rows), 3)
           for k in ("scan", "hash", "scan_span", "hash_span", "scan_mhz", "hash_mhz")}
    med.update(grid=min(grid or 256, 256), same_segments=(d == digest),
               scanned_bytes=c.last_scan_bytes())
    med["scan_gb_s"] = round(med["scanned_bytes"] / med["scan_span"] / 1e6, 1)
    med["scan_b_per_cu_cycle"] = round(med["scanned_bytes"] / (med["scan_span"] * 1e-3) /
                                       (med["grid"] * med["scan_mhz"] * 1e6), 3)
    print(json.dumps(med), flush=True)
