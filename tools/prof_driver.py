"""Profiling driver: the bench workload (1024 x 4 MiB, resident in HBM) through N scans.
Run under rocprofv3 (counters for one kernel via --kernel-include-regex)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pfs_amd.cdc import ChunkParams, Chunker  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
files = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
fbytes = int(sys.argv[3]) if len(sys.argv) > 3 else 4 << 20
offs = np.arange(files + 1, dtype=np.uint64) * np.uint64(fbytes)
c = Chunker(ChunkParams(), 0)
data = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
c.fill_synthetic(data, offs, 0xC2)
for _ in range(n):
    r = c.scan(data, offs)
print("segments", len(r.segments), c.timings())
