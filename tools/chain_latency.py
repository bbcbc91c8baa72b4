"""Serial BLAKE2b chain speed (development tool): n independent segments of `size` bytes
hashed in one launch (pfscdc_hash_ranges); one quad per segment, so n <= 16 stay in one
wave and n <= 1024 x 16 put at most one wave per SIMD.  Prints MB/s per chain and SIMD
cycles per 128-B block at the given clock."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pfs_amd.cdc import ChunkParams, Chunker  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
ghz = float(sys.argv[2]) if len(sys.argv) > 2 else 2.4
counts = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 16, 256, 4096]
ch = Chunker(ChunkParams())
for n in counts:
    data = torch.empty(n * size, dtype=torch.uint8, device="cuda")
    ch.fill_synthetic(data, [0, n * size], 7)
    begins = np.arange(n, dtype=np.uint64) * np.uint64(size)
    sizes = np.full(n, size, dtype=np.uint64)
    ch.hash_ranges(data, begins, sizes)  # warm
    ms = []
    for _ in range(3):
        t0 = time.perf_counter()
        ch.hash_ranges(data, begins, sizes)
        ms.append((time.perf_counter() - t0) * 1e3)
    m = min(ms)
    blocks = size / 128
    print(f"{n:5d} chains x {size >> 20} MiB: {m:8.2f} ms  {size / m / 1e3:7.1f} MB/s per chain  "
          f"{m * 1e-3 * ghz * 1e9 / blocks:7.0f} cycles per block @{ghz} GHz", flush=True)
    del data
    torch.cuda.empty_cache()
