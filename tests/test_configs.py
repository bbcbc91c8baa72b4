"""BASELINE.json configs[2..4] at test sizes: the single long stream (c3), the file-sharded
commit (c4) and the dedup-heavy commit (c5), through the same code bench.py runs.

CPU tests pin the dedup generators' host mirror and the hit-rate accounting against the
oracle; GPU tests check the device generators against the mirror and the HIP path against
the C oracle (bit-exact records, equal hit rates)."""
import numpy as np
import pytest

import bench
from oracle import chunker as Ch
from oracle import coracle
from pfs_amd import distributed as pd
from pfs_amd.cdc import (SYNTH_DEDUP_BLOCKS, SYNTH_DEDUP_FILES, SYNTH_RANDOM, ChunkParams,
                         Chunker, synthetic_bytes)

DEFAULT = Ch.Params()
MIB = 1 << 20


def offsets(sizes):
    o = np.zeros(len(sizes) + 1, dtype=np.uint64)
    o[1:] = np.cumsum(np.asarray(sizes, dtype=np.uint64))
    return o


# ---------------------------------------------------------------- CPU: generators, hit rate

def test_dedup_blocks_repeat_pooled_blocks():
    offs = offsets([16 * MIB, 16 * MIB])
    d = synthetic_bytes(offs, 0xC5, SYNTH_DEDUP_BLOCKS)
    blocks = [d[i * MIB:(i + 1) * MIB].tobytes() for i in range(32)]
    assert len(set(blocks)) < 32, "no pooled block repeated"
    assert len(set(blocks)) > 4, "almost everything pooled"
    # non-pooled blocks equal the plain generator's bytes at the same place
    plain = synthetic_bytes(offs, 0xC5, SYNTH_RANDOM)
    same = sum(blocks[i] == plain[i * MIB:(i + 1) * MIB].tobytes() for i in range(32))
    assert 4 < same < 28


def test_dedup_files_repeat_pooled_files():
    sizes = [3 * MIB + 5] * 40
    offs = offsets(sizes)
    d = synthetic_bytes(offs, 7, SYNTH_DEDUP_FILES)
    files = {d[int(offs[f]):int(offs[f + 1])].tobytes() for f in range(40)}
    assert 10 < len(files) < 40


def test_hit_rate_counts_repeats_in_commit_order():
    dt = coracle.SEG_DTYPE
    idx = np.zeros(5, dtype=dt)
    idx["size"] = [10, 20, 30, 40, 50]
    idx["hash"][:, 0] = [1, 2, 1, 3, 2]
    r = bench.hit_rate(idx)
    assert r["segments"] == 5 and r["unique_digests"] == 3
    assert r["segment_hit_rate"] == pytest.approx(2 / 5, abs=1e-5)
    assert r["byte_hit_rate"] == pytest.approx((30 + 50) / 150, abs=1e-5)


def test_oracle_hit_rate_whole_file_dedup():
    sizes = [300 * 1024 + 17] * 200  # ~100 pooled files drawn from 64: many repeats
    offs = offsets(sizes)
    p = Ch.Params(average_bits=16, seed=1, min=32 * 1024, max=128 * 1024)
    d = synthetic_bytes(offs, 9, SYNTH_DEDUP_FILES)
    segs, _ = coracle.segment_files(d, offs, p, nthreads=8)
    r = bench.hit_rate(segs)
    assert r["segment_hit_rate"] > 0.2  # duplicated files give identical segment lists


def test_c4_layout_and_shards():
    # c4 = the commit as pachd serializes it: whole filesets per rank, pieces tile every file
    args = type("A", (), {"config": "c4", "seed": -1, "dedup": "blocks", "group": 1,
                          "mem_threshold": 10 ** 9})()
    total = 0
    ranges = []
    for rank in range(8):
        w = bench.workload(args, 8, rank)
        assert w.scaling == "strong" and w.mode == SYNTH_RANDOM and w.seed == 0xC4
        ranges.append((w.gbase, w.gbase + len(w.sizes)))
        total += w.total
        assert np.array_equal(w.gid, np.arange(*ranges[-1]))
    assert total == 100 * (1 << 30)
    lay = w.layout
    assert ranges[0][0] == 0 and ranges[-1][1] == lay.npieces
    assert all(a[1] == b[0] for a, b in zip(ranges, ranges[1:]))
    assert lay.nfilesets == 108  # 100 GiB / 1e9 B


def test_auto_group_holds_20k_chains():
    args = type("A", (), {"config": "c4", "seed": -1, "dedup": "blocks", "group": 0,
                          "mem_threshold": 10 ** 9})()
    assert bench.workload(args, 1, 0).group == 1  # ~20K chains in one commit
    w8 = bench.workload(args, 8, 3)
    assert w8.group == 8 and w8.total <= 180 << 30
    # copy g holds the same pieces over files g * 10000 + f
    n = w8.per_copy
    assert np.array_equal(w8.ids[n:2 * n], w8.ids[:n] + bench.C4_FILES)
    assert np.array_equal(w8.gid[n:2 * n], w8.gid[:n] + w8.layout.npieces)


# ---------------------------------------------------------------- GPU

gpu = pytest.mark.gpu


@gpu
@pytest.mark.parametrize("mode", [SYNTH_RANDOM, SYNTH_DEDUP_BLOCKS, SYNTH_DEDUP_FILES])
def test_device_generator_modes_match_host(mode):
    import torch
    offs = offsets([3 * MIB + 11, 0, 2 * MIB, 5 * MIB + 1])
    c = Chunker(ChunkParams(), 0)
    t = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
    c.fill_synthetic(t, offs, 0xC5, mode)
    assert np.array_equal(t.cpu().numpy(), synthetic_bytes(offs, 0xC5, mode))


@gpu
def test_shard_fill_keeps_global_file_ids():
    # a rank's pieces of a commit cut into filesets hold exactly the commit's bytes there
    import torch
    sizes = [bench.C4_FILE_BYTES // 8] * 12
    offs = offsets(sizes)
    c = Chunker(ChunkParams(), 0)
    whole = synthetic_bytes(offs, 0xC4, SYNTH_DEDUP_BLOCKS)
    lay = pd.commit_layout(sizes, 3_000_000)
    po = lay.offsets()
    for rng in pd.shard_filesets(lay, 3):
        p0, p1 = pd.rank_pieces(lay, rng)
        w = bench.Work(lay.size[p0:p1], lay.file[p0:p1], lay.start[p0:p1], 0xC4,
                       SYNTH_DEDUP_BLOCKS, {}, "strong", gbase=p0)
        t = torch.empty(max(w.total, 1), dtype=torch.uint8, device="cuda:0")
        bench.fill(c, t, w)
        assert np.array_equal(t[:w.total].cpu().numpy(), whole[int(po[p0]):int(po[p1])])


@gpu
def test_c3_long_single_stream_matches_oracle():
    # one 768 MiB stream, device-resident: block-parallel scan over ~280 tiles stitched into
    # the serial cut set (forced 20 MB cuts included)
    import torch
    offs = offsets([768 * MIB])
    c = Chunker(ChunkParams(), 0)
    t = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
    c.fill_synthetic(t, offs, 0xC3)
    res = c.scan(t, offs)
    segs, begin = coracle.segment_files(t.cpu().numpy(), offs, DEFAULT)
    assert len(res.segments) == len(segs) > 80
    for f in ("offset", "size", "file", "flags", "hash"):
        assert np.array_equal(res.segments[f], segs[f]), f


@gpu
@pytest.mark.parametrize("mode", [SYNTH_DEDUP_BLOCKS, SYNTH_DEDUP_FILES])
def test_c5_dedup_commit_matches_oracle_and_hit_rate(mode):
    import torch
    sizes = [bench.C4_FILE_BYTES] * 32
    offs = offsets(sizes)
    c = Chunker(ChunkParams(), 0)
    t = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
    c.fill_synthetic(t, offs, 0xC5, mode)
    res = c.scan(t, offs)
    segs, _ = coracle.segment_files(t.cpu().numpy(), offs, DEFAULT, nthreads=16)
    for f in ("offset", "size", "file", "flags", "hash"):
        assert np.array_equal(res.segments[f], segs[f]), f
    assert bench.hit_rate(res.segments) == bench.hit_rate(segs)
    if mode == SYNTH_DEDUP_FILES:
        host = t.cpu().numpy()
        distinct = len({host[int(offs[f]):int(offs[f + 1])].tobytes() for f in range(len(sizes))})
        if distinct < len(sizes):  # some pooled file drawn twice -> its segments repeat
            assert bench.hit_rate(res.segments)["segment_hit_rate"] > 0


def test_commit_layout_matches_oracle_unordered_writer():
    # bench.commit_layout = the fileset pieces oracle.fileset.UnorderedWriter produces
    from oracle import fileset as OF
    for sizes, thr in [([300, 500, 200, 0, 1000], 400), ([400, 400, 1], 400), ([5, 0, 7], 100),
                       ([1000], 250)]:
        pieces, streams = bench.commit_layout(sizes, thr)
        uw = OF.UnorderedWriter(DEFAULT, thr)
        uw.serialize = lambda uw=uw: (uw.filesets.append(
            [len(b) for _, _, b in uw.buffer.walk_additive()]) if not uw.buffer.empty() else None,
            setattr(uw, "buffer", OF.Buffer()), setattr(uw, "mem_available", uw.mem_threshold))
        for i, n in enumerate(sizes):
            uw.put(f"/f{i:04d}", "", True, bytes(n))
        uw.serialize()
        want = uw.filesets
        got = [pieces[a:b] for a, b in zip(streams[:-1], streams[1:])]
        assert got == want, (sizes, thr)
