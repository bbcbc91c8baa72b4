"""Multi-rank logic on CPU (gloo, world_size 2, 3, 4 and 8): every sharded form of the path
produces exactly the single-process result.  On the GPU box the same code runs over RCCL
("nccl" backend) from bench.py; here the per-rank compute is the CPU oracle standing in for
the GPU (the sharding, the collectives and the border copies are what is under test).

* independent files: file sharding + the chunk-ref index all-gather;
* a commit: whole serialized filesets per rank (fileset/unordered_writer.go:45-122), each
  rank its own UnorderedWriter over its pieces; the gathered filesets (SizeBytes, root
  indexes, every level-0 index entry) equal one writer's over the whole commit;
* one stream: equal byte ranges + halo, gathered candidates, serial select, point-to-point
  copies of straddling segments' bytes; the gathered segments equal one scan's.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import chunker as Ch
from oracle import coracle
from oracle import fileset as OF
from pfs_amd import distributed as pd
from pfs_amd.cdc import synthetic_bytes, synthetic_piece_bytes

P = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
SMALL_INDEX = Ch.Params(average_bits=13, seed=0, min=3000, max=60000)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(target, world, *args):
    """Run target(rank, world, q, *args) in `world` gloo ranks; returns what rank 0 put."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_entry, args=(target, r, world, port, q) + args)
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


def _rank_entry(target, rank, world, port, q, *args):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = target(rank, world, *args)
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


# ---------------------------------------------------------------- independent files

def _workload():
    rng = np.random.default_rng(12)
    lens = rng.integers(0, 80_000, 37)
    lens[5] = 0
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return lens, offs, synthetic_bytes(offs, 12)


def _files_rank(rank, world):
    lens, offs, data = _workload()
    b, e = pd.shard_files(lens, world)[rank]
    loffs = offs[b:e + 1] - offs[b]
    ldata = data[int(offs[b]):int(offs[e])]
    segs, _ = coracle.segment_files(ldata, loffs, P)
    cap = pd.max_segments(lens, P.min)  # one global bound works for every rank
    return pd.gather_index(segs, b, cap).tobytes()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_index_equals_single_process(world):
    from pfs_amd import _lib

    got = np.frombuffer(_spawn(_files_rank, world), dtype=_lib.segment_dtype())
    _, offs, data = _workload()
    want, _ = coracle.segment_files(data, offs, P)
    assert len(got) == len(want)
    for f in ("offset", "size", "file", "flags", "hash"):
        assert np.array_equal(got[f], want[f]), f


def _files_rank_root(rank, world):
    """The bench's per-step gather: live records to rank 0 only (counts first)."""
    lens, offs, data = _workload()
    b, e = pd.shard_files(lens, world)[rank]
    if rank == world - 1:
        e = b  # a rank with no records at all sends nothing
    loffs = offs[b:e + 1] - offs[b]
    ldata = data[int(offs[b]):int(offs[e])]
    segs, _ = coracle.segment_files(ldata, loffs, P)
    st = {}
    got = pd.gather_index_to_root(segs, b, stats=st)
    if rank != 0:
        assert got is None and not st
        return None
    return got.tobytes(), st, (b, e)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_gather_index_to_root_moves_live_records_only(world):
    from pfs_amd import _lib

    raw, st, _ = _spawn(_files_rank_root, world)
    got = np.frombuffer(raw, dtype=_lib.segment_dtype())
    lens, offs, data = _workload()
    last_b = pd.shard_files(lens, world)[world - 1][0]  # the last rank's files are dropped
    want, _ = coracle.segment_files(data[:int(offs[last_b])], offs[:last_b + 1], P)
    assert len(got) == len(want) == st["records"]
    for f in ("offset", "size", "file", "flags", "hash"):
        assert np.array_equal(got[f], want[f]), f
    # rank 0 received exactly the other ranks' live records, no padding
    r0 = pd.shard_files(lens, world)[0]
    own, _ = coracle.segment_files(data[:int(offs[r0[1]])], offs[:r0[1] + 1], P)
    assert st["bytes_received"] == (len(want) - len(own)) * _lib.segment_dtype().itemsize


def _records_root(rank, world):
    recs = np.arange(rank * 3, dtype=np.int64) + 100 * rank  # rank 0: none
    out = pd.gather_records_to_root(recs, dst=world - 1)
    return out if rank == world - 1 else None


def test_gather_records_to_other_root():
    # the root need not be rank 0 (the helper's dst), and rank 0 may hold nothing
    got = _spawn(_records_root_via0, 3)
    want = np.concatenate([np.arange(r * 3, dtype=np.int64) + 100 * r for r in range(3)])
    assert np.array_equal(got, want)


def _records_root_via0(rank, world):
    import torch.distributed as dist
    out = _records_root(rank, world)
    # hand rank 2's result to rank 0 (the spawn helper returns rank 0's value)
    blob = torch.from_numpy(out if out is not None else np.zeros(0, np.int64))
    n = torch.tensor([blob.numel()])
    dist.broadcast(n, src=world - 1)
    buf = blob if rank == world - 1 else torch.empty(int(n.item()), dtype=torch.int64)
    dist.broadcast(buf, src=world - 1)
    return buf.numpy()


def test_shard_files_balanced_and_contiguous():
    rng = np.random.default_rng(0)
    sizes = rng.integers(0, 10_000_000, 1000)
    for w in (1, 2, 4, 8):
        sh = pd.shard_files(sizes, w)
        assert sh[0][0] == 0 and sh[-1][1] == len(sizes)
        assert all(sh[i][1] == sh[i + 1][0] for i in range(w - 1))
        per = [int(sizes[b:e].sum()) for b, e in sh]
        assert max(per) - min(per) <= 2 * int(sizes.max())


def test_pack_unpack_roundtrip():
    from pfs_amd import _lib

    dt = _lib.segment_dtype()
    segs = np.zeros(3, dtype=dt)
    segs["file"] = [0, 0, 1]
    segs["size"] = [5, 6, 7]
    blk = np.concatenate([pd.pack_index(segs, 10, 4), pd.pack_index(segs[:1], 20, 4)])
    out = pd.unpack_index(blk, 2, 4)
    assert list(out["file"]) == [10, 10, 11, 20] and list(out["size"]) == [5, 6, 7, 5]


# ---------------------------------------------------------------- a commit (serialized filesets)

MEM = 120_000


def _commit_sizes():
    rng = np.random.default_rng(21)
    sizes = [int(x) for x in rng.integers(0, 45_000, 40)]
    sizes[3] = 0
    sizes[7] = 200_000  # spans two filesets
    # make file 12 end exactly at a fileset border (io.CopyN exact fill: an empty re-Add)
    lay = pd.commit_layout(sizes[:12], MEM)
    used = int(lay.fileset_bytes()[-1]) if lay.nfilesets else 0
    sizes[11] += MEM - used
    return sizes


def _path(f):
    return "/%016d" % f


def _bytes(f, start, size):
    return synthetic_piece_bytes(f, start, size, 0xC4).tobytes()


def test_commit_layout_pieces():
    sizes = _commit_sizes()
    lay = pd.commit_layout(sizes, MEM)
    assert lay.size.sum() == sum(sizes)
    fb = lay.fileset_bytes()
    assert (fb[:-1] == MEM).all() and 0 < fb[-1] <= MEM
    # every file's pieces are contiguous and start where the previous piece ended
    for f in range(len(sizes)):
        idx = np.nonzero(lay.file == f)[0]
        assert int(lay.start[idx[0]]) == 0 and not lay.append[idx[0]]
        ends = lay.start[idx] + lay.size[idx]
        assert (lay.start[idx[1:]] == ends[:-1]).all() and lay.append[idx[1:]].all()
        assert int(ends[-1]) == sizes[f]
    # the exact fill leaves an empty continuation piece at the start of the next fileset
    k = int(np.nonzero((lay.file == 11) & lay.append & (lay.size == 0))[0][0])
    assert k in set(int(x) for x in lay.fileset_begin)


def _commit_rank(rank, world, index_params):
    sizes = _commit_sizes()
    lay = pd.commit_layout(sizes, MEM)
    rng = pd.shard_filesets(lay, world)[rank]
    w = OF.UnorderedWriter(P, MEM, index_params)
    prims = pd.put_rank_filesets(w, lay, rng, _path, _bytes)
    out = pd.gather_primitives(prims)
    # the level-0 index entries of every fileset (DataRefs with chunk Refs), in commit order
    frames = [b"".join(e[2] for e in log if e[0] == "index") for log in w.log]
    frames = frames[:rng[1] - rng[0]]
    return out, pd.gather_blobs(frames)


@pytest.mark.parametrize("world", [2, 3])
def test_commit_sharded_by_fileset_equals_single_writer(world):
    got, got_frames = _spawn(_commit_rank, world, SMALL_INDEX)
    sizes = _commit_sizes()
    w = OF.UnorderedWriter(P, MEM, SMALL_INDEX)
    for f, n in enumerate(sizes):
        w.put(_path(f), "", False, _bytes(f, 0, n))
    want = w.close()
    assert len(want) >= 4 and len(got) == len(want)
    for i, (g, x) in enumerate(zip(got, want)):
        assert g == (x.additive, x.deletive, x.size_bytes), i
    want_frames = [b"".join(e[2] for e in log if e[0] == "index") for log in w.log]
    assert got_frames == want_frames


def test_commit_sharded_reference_index_params():
    # the reference's own index chunking (avgBits 20, seed = level), world 2
    got, _ = _spawn(_commit_rank, 2, None)
    sizes = _commit_sizes()
    w = OF.UnorderedWriter(P, MEM)
    for f, n in enumerate(sizes):
        w.put(_path(f), "", False, _bytes(f, 0, n))
    want = [(x.additive, x.deletive, x.size_bytes) for x in w.close()]
    assert got == want


def _pieces_rank(rank, world):
    """configs[3] put path: the segments of this rank's pieces (CDC + DataRef hashes per
    piece: every piece is its own annotation), gathered with global piece ids."""
    sizes = _commit_sizes()
    lay = pd.commit_layout(sizes, MEM)
    p0, p1 = pd.rank_pieces(lay, pd.shard_filesets(lay, world)[rank])
    offs = lay.offsets()
    data = np.concatenate([synthetic_piece_bytes(int(lay.file[i]), int(lay.start[i]),
                                                 int(lay.size[i]), 0xC4) for i in range(p0, p1)]
                          or [np.zeros(0, np.uint8)])
    segs, _ = coracle.segment_files(data, offs[p0:p1 + 1] - offs[p0], P)
    return pd.gather_index(segs, p0, pd.max_segments(lay.size, P.min)).tobytes()


@pytest.mark.parametrize("world", [2, 3])
def test_commit_pieces_segments_equal_single(world):
    from pfs_amd import _lib

    got = np.frombuffer(_spawn(_pieces_rank, world), dtype=_lib.segment_dtype())
    lay = pd.commit_layout(_commit_sizes(), MEM)
    data = np.concatenate([synthetic_piece_bytes(int(lay.file[i]), int(lay.start[i]),
                                                 int(lay.size[i]), 0xC4)
                           for i in range(lay.npieces)])
    want, _ = coracle.segment_files(data, lay.offsets(), P)
    assert len(got) == len(want)
    for f in ("offset", "size", "file", "flags", "hash"):
        assert np.array_equal(got[f], want[f]), f


# ---------------------------------------------------------------- one stream split across ranks

def _stream(kind):
    n = 2_500_000
    data = synthetic_bytes([0, n], 0xC3)
    if kind == "zeros":  # no candidates inside the run: forced cuts at max across borders
        data[600_000:1_900_000] = 0
    return data


def _cands_oracle(t, halo):
    c = coracle.candidates(t.numpy(), P)
    return c[c >= halo]


def _hash_oracle(t, begins, sizes):
    a = t.numpy()
    return np.stack([np.frombuffer(hashlib.blake2b(a[int(b):int(b) + int(s)].tobytes(),
                                                   digest_size=32).digest(), np.uint8)
                     for b, s in zip(begins, sizes)])


def _stream_rank(rank, world, kind):
    data = _stream(kind)
    n = len(data)
    a, b = pd.split_stream(n, world)[rank]
    halo = min(a, 64)
    local = torch.zeros(halo + (b - a) + P.max, dtype=torch.uint8)
    local[:halo + b - a] = torch.from_numpy(data[a - halo:b].copy())
    segs = pd.stream_segments(local, n, (a, b), halo, P.min, P.max, _cands_oracle, _hash_oracle)
    return segs.tobytes()


@pytest.mark.parametrize("world,kind", [(2, "random"), (3, "random"), (3, "zeros"),
                                        (8, "random"), (8, "zeros")])
def test_split_stream_equals_single_scan(world, kind):
    from pfs_amd import _lib

    got = np.frombuffer(_spawn(_stream_rank, world, kind), dtype=_lib.segment_dtype())
    data = _stream(kind)
    want, _ = coracle.segment_files(data, [0, len(data)], P)
    assert len(got) == len(want) and len(want) > 50
    for f in ("offset", "size", "flags", "hash"):
        assert np.array_equal(got[f], want[f]), f
    if kind == "zeros":
        assert (want["size"] == P.max).sum() >= 10  # forced cuts straddle the borders
    # the bench's own check of a split stream's line (benchkit.parity) passes on it
    from benchkit import parity
    from pfs_amd.cdc import ChunkParams
    ranges = pd.split_stream(len(data), world)
    seed = 0xC3
    r = parity.stream_border_parity(got, len(data), ranges, seed,
                                    ChunkParams(P.average_bits, P.seed, P.min, P.max))
    if kind == "random":  # (the zeros run is not the synthetic stream the check regenerates)
        assert r["gpu_equals_cpu_oracle"] and r["border_segments_checked"] >= world - 1


def test_select_cuts_equals_oracle():
    rng = np.random.default_rng(3)
    for _ in range(20):
        n = int(rng.integers(0, 400_000))
        cands = np.unique(rng.integers(63, max(n, 64), int(rng.integers(0, 60))))
        cands = cands[cands < n]
        offs, sizes, flags = pd.select_cuts(cands, n, P.min, P.max)
        cuts = Ch.select_cuts(n, cands, P)
        assert [int(o + s - 1) for o, s, f in zip(offs, sizes, flags) if f & 2] == cuts
        assert int(sizes.sum()) == n


def test_put_rank_filesets_every_split_point():
    # every fileset border as the rank border, including the one right after the exact fill
    # (whose trailing local fileset must be dropped): the concatenation equals one writer
    sizes = _commit_sizes()
    lay = pd.commit_layout(sizes, MEM)
    w = OF.UnorderedWriter(P, MEM, SMALL_INDEX)
    for f, n in enumerate(sizes):
        w.put(_path(f), "", False, _bytes(f, 0, n))
    want = [(x.additive, x.deletive, x.size_bytes) for x in w.close()]
    exact = [k for k in range(1, lay.nfilesets)
             if lay.append[lay.fileset_begin[k]] and lay.size[lay.fileset_begin[k]] == 0]
    assert exact, "the workload has no exact fill at a fileset border"
    for k in range(1, lay.nfilesets):
        got = []
        for rng in ((0, k), (k, lay.nfilesets)):
            ow = OF.UnorderedWriter(P, MEM, SMALL_INDEX)
            got += [(x.additive, x.deletive, x.size_bytes)
                    for x in pd.put_rank_filesets(ow, lay, rng, _path, _bytes)]
        assert got == want, k
