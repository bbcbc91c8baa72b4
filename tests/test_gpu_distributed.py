"""GPU side of the multi-GPU forms (pfs_amd/distributed.py), on the one GPU of the box:

* the split-stream primitives (pfscdc_candidates over ranges with a halo, host selection,
  pfscdc_hash_ranges) reproduce one pfscdc_scan of the whole stream, dense tiles included;
* the commit sharded by serialized fileset: per-"rank" GPU UnorderedWriters over the rank's
  pieces give the filesets of one GPU writer (and of the oracle);
* a single-rank RCCL ("nccl") process group runs the device-tensor gathers and the
  split-stream driver, so the backend the bench uses at N > 1 has run on the hardware.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import fuzz_cases
import torch

from oracle import chunker as Ch
from oracle import coracle
from oracle import fileset as OF
from pfs_amd import distributed as pd
from pfs_amd import fileset as PF
from pfs_amd.cdc import ChunkParams, Chunker, synthetic_bytes, synthetic_piece_bytes

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

P = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
SMALL_INDEX = Ch.Params(average_bits=13, seed=0, min=3000, max=60000)


def cp(p):
    return ChunkParams(p.average_bits, p.seed, p.min, p.max)


def split_scan(ch, dev, n, world, params):
    """The split-stream algorithm with `world` virtual ranks on one GPU (no collectives)."""
    cands = []
    for a, b in pd.split_stream(n, world):
        halo = min(a, 64)
        # each rank's buffer starts 16-B aligned: copy its halo + range
        loc = dev[a - halo:b].clone()
        cands.append(ch.candidates(loc, halo).astype(np.uint64) + np.uint64(a - halo))
    cands = np.concatenate(cands)
    offs, sizes, flags = pd.select_cuts(cands, n, params.min, params.max)
    digests = ch.hash_ranges(dev, offs, sizes)
    return cands, offs, sizes, flags, digests


@pytest.mark.parametrize("world", [1, 2, 5])
def test_split_stream_primitives_equal_scan(world):
    n = 7_000_003
    data = synthetic_bytes([0, n], 0xC3)
    data[2_000_000:3_100_000] = 0  # forced cuts at max across a border
    dev = torch.from_numpy(data).cuda()
    ch = Chunker(cp(P))
    cands, offs, sizes, flags, digests = split_scan(ch, dev, n, world, P)
    assert np.array_equal(cands, coracle.candidates(data, P, cap=1 << 22))
    res = ch.scan(dev, [0, n])
    segs = res.segments
    assert len(segs) == len(offs) > 100
    assert np.array_equal(segs["offset"], offs) and np.array_equal(segs["size"], sizes)
    assert np.array_equal(segs["flags"], flags)
    assert np.array_equal(segs["hash"], digests)
    ch.close()


@pytest.mark.parametrize("case", fuzz_cases(6))
def test_split_stream_random_borders_equal_scan(case):
    """Randomised single streams split over 1-8 virtual ranks: length, parameters and
    constant runs (candidates everywhere or nowhere, forced cuts) drawn per case; the
    gathered candidates equal the oracle's, and the selected segments and digests one scan's."""
    rng = np.random.default_rng(5500 + case)
    n = int(rng.integers(300_000, 9_000_000))
    bits = int(rng.integers(9, 15))
    mn = int(rng.integers(64, 8000))
    p = Ch.Params(average_bits=bits, seed=int(rng.integers(0, 3)), min=mn,
                  max=mn + int(rng.integers(1, 8 * (1 << bits))))
    world = int(rng.integers(1, 9))
    data = synthetic_bytes([0, n], 600 + case)
    for _ in range(int(rng.integers(0, 4))):
        a = int(rng.integers(0, n))
        data[a:a + int(rng.integers(1, 400_000))] = int(rng.integers(0, 256))
    dev = torch.from_numpy(data).cuda()
    ch = Chunker(cp(p))
    cands, offs, sizes, flags, digests = split_scan(ch, dev, n, world, p)
    assert np.array_equal(cands, coracle.candidates(data, p, cap=1 << 24))
    segs = ch.scan(dev, [0, n]).segments
    assert np.array_equal(segs["offset"], offs) and np.array_equal(segs["size"], sizes)
    assert np.array_equal(segs["flags"], flags)
    assert np.array_equal(segs["hash"], digests)
    ch.close()


def test_candidates_dense_tiles_and_halo():
    # avgBits 3: ~1 candidate per 8 bytes, every tile dense (re-rolled on the host)
    p = Ch.Params(average_bits=3, seed=1, min=64, max=5000)
    n = 4_000_000
    data = synthetic_bytes([0, n], 5)
    dev = torch.from_numpy(data).cuda()
    ch = Chunker(cp(p))
    want = coracle.candidates(data, p, cap=1 << 22)
    assert len(want) > 100_000
    got = np.concatenate([ch.candidates(dev[a - min(a, 64):b].clone(), min(a, 64))
                          + np.uint64(a - min(a, 64)) for a, b in pd.split_stream(n, 3)])
    assert np.array_equal(got, want)
    ch.close()


def test_hash_ranges_host_and_device():
    data = synthetic_bytes([0, 1_000_000], 77)
    ch = Chunker(cp(P))
    begins = np.array([0, 5, 1000, 999_999, 123_456], dtype=np.uint64)
    sizes = np.array([0, 1, 128, 1, 300_000], dtype=np.uint64)
    want = np.stack([np.frombuffer(Ch.blake2b256(data[int(b):int(b + s)].tobytes()), np.uint8)
                     for b, s in zip(begins, sizes)])
    assert np.array_equal(ch.hash_ranges(data, begins, sizes), want)
    assert np.array_equal(ch.hash_ranges(torch.from_numpy(data).cuda(), begins, sizes), want)
    ch.close()


def test_fill_synthetic_pieces_matches_host():
    ch = Chunker(cp(P))
    pieces = [(3, 0, 1000), (3, 1000, 77), (9, 123_457, 50_001), (0, 0, 0), (12, 5, 8)]
    offs = np.concatenate([[0], np.cumsum([s for _, _, s in pieces])]).astype(np.uint64)
    t = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda")
    for mode in (0, 1, 2):
        ch.fill_synthetic_pieces(t, offs, [f for f, _, _ in pieces], [s for _, s, _ in pieces],
                                 0xC4, mode)
        want = np.concatenate([synthetic_piece_bytes(f, s, n, 0xC4, mode) for f, s, n in pieces])
        assert np.array_equal(t.cpu().numpy(), want), mode
    ch.close()


MEM = 120_000


def _commit_sizes():
    rng = np.random.default_rng(21)
    sizes = [int(x) for x in rng.integers(0, 45_000, 40)]
    sizes[3] = 0
    sizes[7] = 200_000
    lay = pd.commit_layout(sizes[:12], MEM)
    sizes[11] += MEM - int(lay.fileset_bytes()[-1])
    return sizes


def _path(f):
    return "/%016d" % f


def _bytes(f, start, size):
    return synthetic_piece_bytes(f, start, size, 0xC4).tobytes()


@pytest.mark.parametrize("world", [2, 3])
def test_commit_sharded_gpu_writers_equal_single(world):
    sizes = _commit_sizes()
    lay = pd.commit_layout(sizes, MEM)
    st = PF.Storage(0, cp(P), MEM, cp(SMALL_INDEX))
    got = []
    for rng in pd.shard_filesets(lay, world):
        w = st.new_unordered_writer()
        got += [(x.additive, x.deletive, x.size_bytes)
                for x in pd.put_rank_filesets(w, lay, rng, _path, _bytes)]
    one = st.new_unordered_writer()
    for f, n in enumerate(sizes):
        one.put(_path(f), "", False, _bytes(f, 0, n))
    single = [(x.additive, x.deletive, x.size_bytes) for x in one.close()]
    ow = OF.UnorderedWriter(P, MEM, SMALL_INDEX)
    for f, n in enumerate(sizes):
        ow.put(_path(f), "", False, _bytes(f, 0, n))
    want = [(x.additive, x.deletive, x.size_bytes) for x in ow.close()]
    assert single == want
    assert got == want


def test_rccl_single_rank_gathers_and_split_stream():
    # a fresh process: the nccl (RCCL) backend, device tensors, world size 1
    code = r"""
import os, sys
sys.path.insert(0, %r)
import numpy as np, torch, torch.distributed as dist
from oracle import chunker as Ch
from oracle import coracle
from pfs_amd import distributed as pd
from pfs_amd.cdc import ChunkParams, Chunker, synthetic_bytes
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ["PFS_TEST_PORT"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
assert dist.get_backend() == "nccl"
p = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
ch = Chunker(ChunkParams(12, 1, 2000, 30000))
offs = np.array([0, 100_000, 100_001, 357_000, 357_000, 1_000_000], dtype=np.uint64)
data = synthetic_bytes(offs, 42)
res = ch.scan(torch.from_numpy(data).to(dev), offs)
idx = pd.gather_index(res.segments, 0, pd.max_segments(np.diff(offs), p.min), device=dev)
want, _ = coracle.segment_files(data, offs, p)
assert idx.tobytes() == want.tobytes()
assert pd.gather_records(want, device=dev).tobytes() == want.tobytes()
st = {}
assert pd.gather_index_to_root(res.segments, device=dev, stats=st).tobytes() == want.tobytes()
assert st == {"records": len(want), "bytes_received": 0, "count_bytes": 8}
assert pd.gather_records_to_root(want, device=dev).tobytes() == want.tobytes()
assert pd.gather_blobs([b"abc", b"", b"xyz"], device=dev) == [b"abc", b"", b"xyz"]
n = 3_000_000
s = synthetic_bytes([0, n], 0xC3)
local = torch.zeros(n + p.max, dtype=torch.uint8, device=dev)
local[:n] = torch.from_numpy(s).to(dev)
segs = pd.stream_segments(local, n, (0, n), 0, p.min, p.max,
                          lambda t, h: ch.candidates(t, h),
                          lambda t, b, z: ch.hash_ranges(t, b, z), device=dev)
want, _ = coracle.segment_files(s, [0, n], p)
for f in ("offset", "size", "flags", "hash"):
    assert np.array_equal(segs[f], want[f]), f
# the border copy of stream_segments (distributed.py: batch_isend_irecv of device slices of
# `local` into the room after the next range) through RCCL itself: at world size 1 the plan
# has no border, so send a straddling segment's tail to ourselves the same way
tail = local[1_000_000:1_000_000 + p.max]  # a forced max-size segment's worth
room = local[n:n + p.max]
room.zero_()
reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, tail.contiguous(), 0),
                               dist.P2POp(dist.irecv, room, 0)])
for r in reqs:
    r.wait()
torch.cuda.synchronize()
assert torch.equal(room, tail), "RCCL self send/recv of the border bytes"
dist.destroy_process_group()
print("rccl ok", len(segs))
""" % ROOT
    import socket

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    env = dict(os.environ, PFS_TEST_PORT=str(port))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl ok" in r.stdout


# index chunking whose min exceeds any entry here (pieces <= 200 KB of ~4 KB chunks): see
# test_gpu_fileset.RAND_INDEX for why an entry at the index min is excluded
RAND_INDEX = Ch.Params(average_bits=16, seed=0, min=40_000, max=400_000)


@pytest.mark.parametrize("case", fuzz_cases(4))
def test_commit_sharded_random_layouts_equal_single(case):
    """Randomised commits sharded by serialized fileset over 2-6 virtual ranks: file sizes
    (empty, exact fills, files larger than the threshold), threshold and rank count drawn per
    case; the ranks' filesets equal one writer's, which equal the oracle's."""
    rng = np.random.default_rng(5600 + case)
    mem = int(rng.integers(40_000, 200_000))
    sizes = [0 if rng.random() < 0.1 else int(rng.integers(1, int(mem * rng.choice([0.3, 1.0, 2.5]))))
             for _ in range(int(rng.integers(5, 40)))]
    if rng.random() < 0.5:  # an exact fill somewhere
        k = int(rng.integers(0, len(sizes)))
        lay = pd.commit_layout(sizes[:k + 1], mem)
        sizes[k] += mem - int(lay.fileset_bytes()[-1])
    world = int(rng.integers(2, 7))
    lay = pd.commit_layout(sizes, mem)
    st = PF.Storage(0, cp(P), mem, cp(RAND_INDEX))
    got = []
    for r in pd.shard_filesets(lay, world):
        w = st.new_unordered_writer()
        got += [(x.additive, x.deletive, x.size_bytes)
                for x in pd.put_rank_filesets(w, lay, r, _path, _bytes)]
    one = st.new_unordered_writer()
    for f, n in enumerate(sizes):
        one.put(_path(f), "", False, _bytes(f, 0, n))
    single = [(x.additive, x.deletive, x.size_bytes) for x in one.close()]
    assert got == single
    ow = OF.UnorderedWriter(P, mem, RAND_INDEX)
    for f, n in enumerate(sizes):
        ow.put(_path(f), "", False, _bytes(f, 0, n))
    assert single == [(x.additive, x.deletive, x.size_bytes) for x in ow.close()]
