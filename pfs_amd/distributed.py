"""Multi-GPU forms of the ingest path: one process per GPU, ``torch.distributed`` over RCCL
(backend "nccl" on ROCm) for the few exchanges the path has, gloo for the CPU tests.

Three ways the work shards, each exact (every rank's output equals the matching slice of the
single-GPU output):

* **Independent files** (configs[1]): each file is its own chunk stream (a fresh writer and
  one annotation), and the hash and seglen reset at every Annotate
  (/root/reference/src/internal/storage/chunk/writer.go:125-128), so a file's cuts and DataRef
  digests depend on its own bytes only.  Ranks take contiguous file ranges; the one exchange
  is the all-gather of the segment records (the chunk-ref index).
* **A commit** (configs[3], configs[4]): pachd's UnorderedWriter cuts the Put byte stream
  into serialized filesets of memThreshold bytes (fileset/unordered_writer.go:45-72), and
  every serialized fileset is written by a fresh fileset.Writer with a fresh chunk.Writer
  (unordered_writer.go:83-122, fileset/writer.go:36-50).  Chunks span files inside a fileset
  (writer.go:118-130), never across filesets, so ranks take whole filesets: a file cut at a
  fileset border is two pieces, the second one re-Added in the next fileset (append), exactly
  as the global UnorderedWriter does.  Chunks, Refs and index roots are then formed locally
  and gathered.
* **One stream** (configs[2]): equal byte ranges plus a 64-byte halo; candidates gathered,
  the serial min/max selection of writer.go:163-189 run on every rank over the sorted list,
  segments that straddle a border hashed by the rank holding their first byte after a
  point-to-point copy of the neighbour's bytes (RCCL send/recv over xGMI).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional, Sequence

import numpy as np

from . import _lib


# ---------------------------------------------------------------- independent files

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
        target = -(-total * r // world_size)  # ceil, exact (the C ABI's pfscdc_deal)
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


def gather_records(recs: np.ndarray, device=None, group=None) -> np.ndarray:
    """All-gather a variable number of fixed-size records per rank (any numpy dtype), in rank
    order: one all-gather of the counts, one of the blocks padded to the largest count."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    recs = np.ascontiguousarray(recs)
    isz = recs.dtype.itemsize
    cnt = torch.tensor([len(recs)], dtype=torch.int64, device=device)
    cnts = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(cnts, cnt, group=group)
    cnts = cnts.cpu().numpy()
    cap = max(int(cnts.max()), 1)
    blk = np.zeros(cap * isz, dtype=np.uint8)
    blk[:len(recs) * isz] = recs.view(np.uint8).reshape(-1)
    t = torch.from_numpy(blk)
    if device is not None:
        t = t.to(device)
    out = torch.empty(world * t.numel(), dtype=torch.uint8, device=t.device)
    dist.all_gather_into_tensor(out, t, group=group)
    out = out.cpu().numpy().reshape(world, cap * isz)
    parts = [out[r, :int(cnts[r]) * isz].view(recs.dtype) for r in range(world)]
    return np.concatenate(parts) if parts else recs[:0]


def gather_records_to_root(recs: np.ndarray, device=None, group=None, dst: int = 0,
                           stats: Optional[dict] = None) -> Optional[np.ndarray]:
    """Gather a variable number of fixed-size records per rank to rank ``dst`` alone, in rank
    order: one all-gather of the 8-byte counts, then point-to-point sends of exactly each
    rank's live records (RCCL send/recv over xGMI on device tensors, gloo on host tensors).
    This is the chunk-ref index's collection point: one consumer, as fileset.Writer's
    callback collects the DataRefs of every chunk in one place
    (/root/reference/src/internal/storage/fileset/writer.go:127-149).  Nothing is padded and
    no other rank receives anything.  Returns the records on ``dst``, None elsewhere;
    ``stats`` (if given) gets the record count and the bytes ``dst`` received."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    recs = np.ascontiguousarray(recs)
    isz = recs.dtype.itemsize
    cnt = torch.tensor([len(recs)], dtype=torch.int64, device=device)
    cnts = torch.empty(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(cnts, cnt, group=group)
    cnts = cnts.cpu().numpy()

    def peer(r):
        return r if group is None else dist.get_global_rank(group, r)

    if rank != dst:
        if len(recs):
            t = torch.from_numpy(recs.view(np.uint8).reshape(-1))
            if device is not None:
                t = t.to(device)
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, peer(dst), group)]):
                req.wait()
        return None
    others = int(cnts.sum()) - len(recs)
    buf = torch.empty(others * isz, dtype=torch.uint8, device=device)
    ops, views, pos = [], {}, 0
    for r in range(world):
        n = int(cnts[r]) * isz
        if r == dst or n == 0:
            continue
        views[r] = (pos, n)
        ops.append(dist.P2POp(dist.irecv, buf[pos:pos + n], peer(r), group))
        pos += n
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    got = buf.cpu().numpy() if others else np.zeros(0, dtype=np.uint8)
    parts = []
    for r in range(world):
        if r == dst:
            parts.append(recs)
        elif r in views:
            a, n = views[r]
            parts.append(got[a:a + n].view(recs.dtype))
    if stats is not None:
        stats.update({"records": int(cnts.sum()), "bytes_received": others * isz,
                      "count_bytes": 8 * world})
    return np.concatenate(parts) if parts else recs[:0]


def gather_index_to_root(segments: np.ndarray, file_base: int = 0, device=None, group=None,
                         dst: int = 0, stats: Optional[dict] = None) -> Optional[np.ndarray]:
    """The chunk-ref index (segment records with global file ids) of every rank on ``dst``
    only, live records alone (gather_records_to_root); None on the other ranks."""
    segs = np.ascontiguousarray(segments).copy()
    if file_base:
        segs["file"] = (segs["file"].astype(np.uint64) + np.uint64(file_base)).astype(np.uint32)
    return gather_records_to_root(segs, device, group, dst, stats)


def gather_blobs(blobs: Sequence[bytes], device=None, group=None) -> list[bytes]:
    """All-gather each rank's list of byte strings (encoded index roots and the like);
    returns every rank's blobs in rank order."""
    lens = np.asarray([len(b) for b in blobs], dtype=np.int64)
    all_lens = gather_records(lens, device, group)
    data = np.frombuffer(b"".join(blobs), dtype=np.uint8)
    all_data = gather_records(data, device, group).tobytes()
    out, pos = [], 0
    for n in all_lens:
        out.append(all_data[pos:pos + int(n)])
        pos += int(n)
    return out


# ---------------------------------------------------------------- a commit: serialized filesets

@dataclass
class CommitLayout:
    """A commit's files as pachd serializes them: piece i is bytes [start[i], start[i] +
    size[i]) of file ``file[i]``; fileset k is pieces [fileset_begin[k], fileset_begin[k+1]).
    ``append[i]``: the piece continues a file Put into an earlier fileset (the re-Add after a
    serialization, unordered_writer.go:66-69), so it has no delete record of its own."""
    file: np.ndarray
    start: np.ndarray
    size: np.ndarray
    append: np.ndarray
    fileset_begin: np.ndarray

    @property
    def npieces(self) -> int:
        return len(self.size)

    @property
    def nfilesets(self) -> int:
        return len(self.fileset_begin) - 1

    def offsets(self) -> np.ndarray:
        """Byte offsets of the pieces in the concatenated commit stream (npieces + 1)."""
        o = np.zeros(self.npieces + 1, dtype=np.uint64)
        o[1:] = np.cumsum(self.size.astype(np.uint64))
        return o

    def fileset_bytes(self) -> np.ndarray:
        o = self.offsets()
        fb = self.fileset_begin
        return (o[fb[1:]] - o[fb[:-1]]).astype(np.int64)


def commit_layout(file_sizes: Sequence[int], mem_threshold: int) -> CommitLayout:
    """UnorderedWriter.Put of every file in path order (unordered_writer.go:45-72): each Put
    copies io.CopyN(buffer, r, memAvailable) until EOF, serializing the buffer whenever
    memAvailable reaches 0 and re-Adding the same path to the fresh buffer (so a Put that
    fills the threshold exactly leaves an empty piece in the next fileset)."""
    files, starts, sizes, app, begin = [], [], [], [], [0]
    avail = int(mem_threshold)
    for f, n in enumerate(file_sizes):
        n, pos = int(n), 0
        files.append(f), starts.append(0), sizes.append(0), app.append(False)  # buffer.Add
        while True:
            got = min(avail, n - pos)
            sizes[-1] += got
            pos += got
            eof = got < avail
            avail -= got
            if eof:
                break
            if avail == 0:  # serialize, then the re-Add of the same path
                begin.append(len(sizes))
                avail = int(mem_threshold)
                files.append(f), starts.append(pos), sizes.append(0), app.append(True)
    if begin[-1] != len(sizes):  # Close serializes the rest
        begin.append(len(sizes))
    return CommitLayout(np.asarray(files, dtype=np.uint32), np.asarray(starts, dtype=np.uint64),
                        np.asarray(sizes, dtype=np.uint64), np.asarray(app, dtype=bool),
                        np.asarray(begin, dtype=np.int64))


def shard_filesets(layout: CommitLayout, world_size: int) -> list[tuple[int, int]]:
    """Contiguous fileset ranges [begin, end) per rank, balanced by bytes."""
    return shard_files(layout.fileset_bytes(), world_size)


def rank_pieces(layout: CommitLayout, fs_range: tuple[int, int]) -> tuple[int, int]:
    """Pieces [p0, p1) of the filesets [fs_range)."""
    return int(layout.fileset_begin[fs_range[0]]), int(layout.fileset_begin[fs_range[1]])


def rank_puts(layout: CommitLayout, fs_range: tuple[int, int]):
    """The Put calls that make a fresh UnorderedWriter serialize exactly the filesets of
    fs_range: (file id, byte start in the file, size, append) per piece.  Filesets after the
    first start with a fresh buffer and a full memAvailable in the global writer too, and a
    continuation piece is Put with append (no delete record), as the re-Add was."""
    p0, p1 = rank_pieces(layout, fs_range)
    return [(int(layout.file[i]), int(layout.start[i]), int(layout.size[i]), bool(layout.append[i]))
            for i in range(p0, p1)]


def put_rank_filesets(writer, layout: CommitLayout, fs_range: tuple[int, int],
                      path_of: Callable[[int], str], bytes_of: Callable[[int, int, int], bytes]):
    """Put this rank's pieces (rank_puts) into a fresh UnorderedWriter and Close it; returns
    its serialized filesets.  A rank whose last Put fills the threshold exactly leaves the
    re-Added empty path in a further buffer, which the global writer serializes as the start
    of the next rank's first fileset: that trailing local fileset is dropped."""
    for f, start, size, append in rank_puts(layout, fs_range):
        writer.put(path_of(f), "", append, bytes_of(f, start, size))
    return list(writer.close())[:fs_range[1] - fs_range[0]]


def encode_primitive(additive: Optional[bytes], deletive: Optional[bytes], size: int) -> bytes:
    """One serialized fileset as gathered: SizeBytes (int64 LE), then each root index with a
    presence byte and an int64 LE length."""
    out = int(size).to_bytes(8, "little", signed=True)
    for root in (additive, deletive):
        out += (b"\x01" + len(root).to_bytes(8, "little") + root) if root is not None else b"\x00"
    return out


def decode_primitive(b: bytes) -> tuple[Optional[bytes], Optional[bytes], int]:
    size = int.from_bytes(b[:8], "little", signed=True)
    pos, roots = 8, []
    for _ in range(2):
        if b[pos] == 0:
            roots.append(None)
            pos += 1
        else:
            n = int.from_bytes(b[pos + 1:pos + 9], "little")
            roots.append(b[pos + 9:pos + 9 + n])
            pos += 9 + n
    return roots[0], roots[1], size


def gather_primitives(prims, device=None, group=None) -> list:
    """All-gather every rank's filesets (objects with additive, deletive, size_bytes) in rank
    order = commit order: the commit's fileset list, identical to a single writer's."""
    blobs = [encode_primitive(p.additive, p.deletive, p.size_bytes) for p in prims]
    return [decode_primitive(b) for b in gather_blobs(blobs, device, group)]


# ---------------------------------------------------------------- one stream split across ranks

def split_stream(n: int, world_size: int, align: int = 64) -> list[tuple[int, int]]:
    """Equal byte ranges [a, b) of an n-byte stream (borders rounded to ``align``)."""
    bounds = [0] + [min(n, (n * r // world_size) // align * align) for r in range(1, world_size)]
    bounds.append(n)
    for r in range(1, len(bounds)):
        bounds[r] = max(bounds[r], bounds[r - 1])
    return [(bounds[r], bounds[r + 1]) for r in range(world_size)]


def select_cuts(cands: np.ndarray, n: int, min_chunk: int, max_chunk: int):
    """Writer.roll's serial cut rule (writer.go:163-189) over the sorted candidate positions
    of one annotation of n bytes: a segment starting at s ends at the first candidate
    >= s + min - 1, unless s + max - 1 comes first (forced cut); the rest of the stream after
    the last cut is an open tail.  Returns (offset, size, flags) arrays (PFSCDC_SEG_*)."""
    cands = np.asarray(cands, dtype=np.uint64)
    offs, sizes, flags = [], [], []
    s = 0
    while True:
        lo, hi = s + min_chunk - 1, s + max_chunk - 1
        if lo >= n:
            break
        j = int(np.searchsorted(cands, np.uint64(lo), side="left"))
        c = int(cands[j]) if j < len(cands) else None
        cut = c if c is not None and c <= hi else hi
        if cut >= n:
            break
        offs.append(s), sizes.append(cut + 1 - s), flags.append(_lib.SEG_VALID | _lib.SEG_CUT)
        s = cut + 1
    if s < n:
        offs.append(s), sizes.append(n - s), flags.append(_lib.SEG_VALID)
    return (np.asarray(offs, dtype=np.uint64), np.asarray(sizes, dtype=np.uint64),
            np.asarray(flags, dtype=np.uint32))


def stream_segments(local, n: int, rng: tuple[int, int], halo: int, min_chunk: int,
                    max_chunk: int, candidates_fn: Callable, hash_fn: Callable,
                    device=None, group=None) -> np.ndarray:
    """Segments (with BLAKE2b digests) of one n-byte stream split across the ranks of group.

    local: this rank's uint8 torch tensor holding ``halo`` bytes of the previous range, its
      range [a, b) = rng, and room for max_chunk more bytes (the tail of a segment that
      straddles b is received there).
    candidates_fn(tensor, halo) -> sorted candidate offsets into the tensor (>= halo).
    hash_fn(tensor, begins, sizes) -> uint8[k, 32] digests of ranges of the tensor.
    Every rank returns the whole stream's segment records (file 0, offset = stream offset),
    identical to a single-GPU scan of the stream."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    a, b = rng
    if local.numel() < halo + (b - a) + max_chunk:
        raise ValueError("local buffer needs max_chunk bytes of room after the range")
    loc = candidates_fn(local[:halo + (b - a)], halo).astype(np.uint64)
    glob = loc + np.uint64(a - halo)
    cands = gather_records(glob, device, group)  # rank order == stream order: sorted
    offs, sizes, flags = select_cuts(cands, n, min_chunk, max_chunk)
    # every rank knows every rank's range and every segment: plan the border copies
    ranges = gather_records(np.asarray([a, b], dtype=np.int64), device, group).reshape(-1, 2)
    ends = offs + sizes
    # gloo (CPU tests, one-GPU rehearsals) moves host tensors only: stage device bytes
    staged = local.is_cuda and dist.get_backend(group) == "gloo"
    ops = []
    recv_views = []  # (device view, host staging buffer)
    for q in range(world):
        qa, qb = int(ranges[q][0]), int(ranges[q][1])
        own = np.nonzero((offs >= qa) & (offs < qb))[0]
        if len(own) == 0 or int(ends[own[-1]]) <= qb:
            continue
        need_a, need_b = qb, int(ends[own[-1]])  # bytes q needs from the ranks after it
        for p in range(q + 1, world):
            pa, pb = int(ranges[p][0]), int(ranges[p][1])
            lo, hi = max(need_a, pa), min(need_b, pb)
            if lo >= hi:
                continue
            if rank == p:  # send my bytes [lo, hi) to q
                src = local[halo + (lo - a):halo + (hi - a)]
                src = src.cpu() if staged else src.contiguous()
                ops.append(dist.P2POp(dist.isend, src, q, group))
            elif rank == q:  # receive into the room after my range
                dst = local[halo + (lo - a):halo + (hi - a)]
                buf = torch.empty(dst.numel(), dtype=torch.uint8) if staged else dst
                recv_views.append((dst, buf))
                ops.append(dist.P2POp(dist.irecv, buf, p, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        for dst, buf in recv_views:
            if buf is not dst:
                dst.copy_(buf)
    mine = np.nonzero((offs >= a) & (offs < b))[0]
    dt = _lib.segment_dtype()
    recs = np.zeros(len(mine), dtype=dt)
    if len(mine):
        begins = offs[mine] - np.uint64(a) + np.uint64(halo)
        digests = hash_fn(local, begins, sizes[mine])
        recs["offset"] = offs[mine]
        recs["size"] = sizes[mine]
        recs["flags"] = flags[mine]
        recs["hash"] = digests
    return gather_records(recs, device, group)
