"""Per-step kernel times of one config (development tool): python tools/step_times.py c4 8"""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from pfs_amd.cdc import ChunkParams, Chunker  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
args = bench.parse.__wrapped__() if hasattr(bench.parse, "__wrapped__") else None
sys.argv = [sys.argv[0], "--config", cfg]
args = bench.parse()
work = bench.workload(args, 1, 0)
c = Chunker(ChunkParams(), 0)
data = torch.empty(work.total, dtype=torch.uint8, device="cuda:0")
bench.fill(c, data, work)
for k in range(steps):
    c.scan_async(data, work.offs)
    c.wait()
    t = c.timings()
    print(k, {n: round(t[n], 2) for n in ("scan", "hash", "hash_span")}, flush=True)
