"""Multi-rank logic on CPU (gloo, world_size 2 and 3): file sharding and the chunk-ref index
all-gather produce exactly the single-process index.  On the GPU box the same code runs
over RCCL ("nccl" backend) from bench.py; here the per-rank segmentation is the CPU oracle
standing in for the GPU (the collective and packing logic is what is under test)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import chunker as Ch
from oracle import coracle
from pfs_amd import distributed as pd
from pfs_amd.cdc import synthetic_bytes

P = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _workload():
    rng = np.random.default_rng(12)
    lens = rng.integers(0, 80_000, 37)
    lens[5] = 0
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return lens, offs, synthetic_bytes(offs, 12)


def _rank_main(rank, world, port, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lens, offs, data = _workload()
    shards = pd.shard_files(lens, world)
    b, e = shards[rank]
    loffs = offs[b:e + 1] - offs[b]
    ldata = data[int(offs[b]):int(offs[e])]
    segs, _ = coracle.segment_files(ldata, loffs, P)
    cap = pd.max_segments(lens, P.min)  # one global bound works for every rank
    idx = pd.gather_index(segs, b, cap)
    if rank == 0:
        q.put(idx.tobytes())
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_index_equals_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from pfs_amd import _lib

    got = np.frombuffer(got, dtype=_lib.segment_dtype())
    _, offs, data = _workload()
    want, _ = coracle.segment_files(data, offs, P)
    assert len(got) == len(want)
    for f in ("offset", "size", "file", "flags", "hash"):
        assert np.array_equal(got[f], want[f]), f


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
