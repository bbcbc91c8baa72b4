"""Does HBM traffic cost the hash clock?  The same BLAKE2b work (32,768 ranges of 4 MiB, one
launch through pfscdc_hash_ranges) over 32,768 distinct ranges of a 128 GiB buffer (every byte
from HBM) and over ranges that all start in the first W bytes of the buffer (W = 4 MiB:
L2/Infinity-Cache resident; W = 256 MiB: the Infinity Cache's size).  Same instructions; a
shorter launch with cache-resident bytes means the HBM reads cost clock (energy), which a fused
scan + hash (one HBM read per byte instead of two) could get back.  Prints one JSON line per
layout: median wall ms of the call (records to the host included, ~1 ms)."""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pfs_amd.cdc import ChunkParams, Chunker  # noqa: E402

n, fb, reps = 32768, 4 << 20, int(sys.argv[1]) if len(sys.argv) > 1 else 5
c = Chunker(ChunkParams(), 0)
data = torch.empty(n * fb, dtype=torch.uint8, device="cuda:0")
c.fill_synthetic(data, np.arange(n + 1, dtype=np.uint64) * np.uint64(fb), 0xC2)
torch.cuda.synchronize()
sizes = np.full(n, fb, dtype=np.uint64)
layouts = {"hbm_distinct": np.arange(n, dtype=np.uint64) * np.uint64(fb),
           "window_256MiB": (np.arange(n, dtype=np.uint64) % np.uint64(64)) * np.uint64(fb),
           "window_4MiB": np.zeros(n, dtype=np.uint64)}
order = list(layouts) + list(layouts)
res = {k: [] for k in layouts}
for name in order:
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        c.hash_ranges(data, layouts[name], sizes)
        res[name].append((time.perf_counter() - t) * 1e3)
for k, v in res.items():
    print(json.dumps({"layout": k, "ms_median": round(statistics.median(v[1:]), 2),
                      "ms_all": [round(x, 2) for x in v]}), flush=True)
