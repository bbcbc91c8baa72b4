"""Multi-GPU form of the ingest path: files of a commit sharded by file across ranks (one
process per GPU), one collective to gather the chunk-ref index.

Why sharding by file is exact: the rolling hash and seglen reset at every Annotate
(/root/reference/src/internal/storage/chunk/writer.go:125-128), so a file's cut positions
and DataRef digests depend only on that file's bytes.  The only exchange the path has is
collecting every file's segment records (the chunk-ref index: file, offset, size, BLAKE2b)
where the fileset index is written (fileset/writer.go:127-149) — an all-gather of
fixed-size padded record blocks over RCCL (backend "nccl" on ROCm), latency-bound and tiny
(56 B per segment).  Cross-file chunk assembly (the buf.Len() >= avg rule) is a cheap serial
scan over those records on the gathering rank (writer.cpp replays the same rule).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from . import _lib


def shard_files(file_sizes: Sequence[int], world_size: int) -> list[tuple[int, int]]:
    """Contiguous file ranges [begin, end) per rank, balanced by bytes (greedy prefix split
    of the path-ordered files into equal-byte parts)."""
    sizes = np.asarray(file_sizes, dtype=np.int64)
    n = len(sizes)
    if world_size < 1:
        raise ValueError("world_size must be >= 1")
    cum = np.concatenate([[0], np.cumsum(sizes)])
    total = int(cum[-1])
    bounds = [0]
    for r in range(1, world_size):
        target = total * r / world_size
        # first file index whose prefix reaches the target, kept monotone
        b = int(np.searchsorted(cum, target, side="left"))
        b = max(bounds[-1], min(b, n))
        bounds.append(b)
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world_size)]


def max_segments(file_sizes: Sequence[int], min_chunk: int) -> int:
    """Upper bound on segments of a set of files (all but a file's last are >= min bytes)."""
    s = np.asarray(file_sizes, dtype=np.int64)
    return int(np.sum(np.where(s > 0, s // min_chunk + 1, 0)))


def pack_index(segments: np.ndarray, file_base: int, cap: int) -> np.ndarray:
    """Fixed-size block: uint64 count, then ``cap`` 56-byte records with global file ids."""
    dt = _lib.segment_dtype()
    n = len(segments)
    if n > cap:
        raise ValueError(f"{n} segments exceed the per-rank capacity {cap}")
    recs = np.zeros(cap, dtype=dt)
    if n:
        recs[:n] = segments
        recs["file"][:n] = segments["file"].astype(np.uint64) + file_base
    head = np.array([n], dtype=np.uint64).view(np.uint8)
    return np.concatenate([head, recs.view(np.uint8)])


def unpack_index(blocks: np.ndarray, world_size: int, cap: int) -> np.ndarray:
    dt = _lib.segment_dtype()
    per = 8 + cap * dt.itemsize
    out = []
    for r in range(world_size):
        b = blocks[r * per:(r + 1) * per]
        n = int(b[:8].view(np.uint64)[0])
        out.append(b[8:].view(dt)[:n])
    return np.concatenate(out) if out else np.zeros(0, dtype=dt)


def gather_index(segments: np.ndarray, file_base: int, cap: int, device=None,
                 group=None) -> Optional[np.ndarray]:
    """All-gather every rank's chunk-ref records (RCCL on GPU tensors, gloo on CPU).

    Returns the global index (ordered by rank = by file, then offset) on every rank."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    block = pack_index(segments, file_base, cap)
    t = torch.from_numpy(block)
    if device is not None:
        t = t.to(device, non_blocking=False)
    out = torch.empty(world * t.numel(), dtype=torch.uint8, device=t.device)
    dist.all_gather_into_tensor(out, t, group=group)
    return unpack_index(out.cpu().numpy(), world, cap)
