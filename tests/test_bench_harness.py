"""The benchmark harness's rules and the N > 1 self-check, on the CPU (benchkit/).

- steps in flight: a timed region holds at least 2 S steps after at least S warmup steps
  (c3's twelve streams were timed over 4 steps, a burst from empty);
- the steady-state window skips the first S completions;
- the parity sample of an N-rank line: the first and last piece of every rank, regenerated
  from (file, offset, seed) on rank 0 and compared with the gathered index;
- the cut-rule check of a split stream's border segments.
"""
import hashlib
import types

import numpy as np
import pytest

from benchkit import harness, parity
from benchkit.common import workload
from oracle import chunker as Ch
from oracle import coracle
from pfs_amd import _lib
from pfs_amd.cdc import (SYNTH_DEDUP_BLOCKS, SYNTH_DEDUP_FILES, SYNTH_RANDOM, ChunkParams,
                         synthetic_bytes, synthetic_piece_bytes)


@pytest.mark.parametrize("steps,warmup,S,want", [
    (10, 3, 1, (10, 3)), (4, 2, 12, (24, 12)), (30, 15, 12, (30, 15)), (1, 0, 2, (4, 2)),
    (5, 1, 2, (5, 2))])
def test_plan_steps(steps, warmup, S, want):
    k, w, note = harness.plan_steps(steps, warmup, S)
    assert (k, w) == want
    assert (note is None) == ((k, w) == (steps, warmup))
    if S > 1:
        assert k >= 2 * S and w >= S


def test_steady_state_skips_the_fill():
    # 12 in flight, completions every 10 ms after a 170 ms fill
    done = [0.170 + 0.010 * i for i in range(24)]
    r = harness.steady_state(0.0, done, 12, 10 << 30)
    assert r["steps"] == 12 and abs(r["ms_per_step"] - 10.0) < 1e-6
    assert abs(r["value"] - 1000.0) < 0.01  # 10 GiB per 10 ms
    assert harness.steady_state(0.0, done[:12], 12, 1) is None


def _args(**kw):
    a = dict(config="c2", files=4, file_bytes=3 << 20, group=2, seed=-1, mem_threshold=10 ** 9,
             dedup="blocks", path="put")
    a.update(kw)
    return types.SimpleNamespace(**a)


def test_sample_pieces_c2_first_and_last_file_of_every_rank():
    a = _args()
    s = parity.sample_pieces(a, 8)
    n = a.files * a.group
    assert [x[1] for x in s] == [g for r in range(8) for g in (r * n, r * n + n - 1)]
    assert all(x[2] == x[1] and x[3] == 0 and x[4] == a.file_bytes for x in s)


def test_sample_pieces_c4_pieces_of_copy0():
    a = _args(config="c4", group=1)
    s = parity.sample_pieces(a, 8)
    assert len(s) == 16
    for r in range(8):
        w = workload(a, 8, r)
        first, last = s[2 * r], s[2 * r + 1]
        assert first[1] == w.gbase and last[1] == w.gbase + w.per_copy - 1
        assert first[4] == w.sizes[0] and last[3] == int(w.starts[w.per_copy - 1])


@pytest.mark.parametrize("mode", [SYNTH_RANDOM, SYNTH_DEDUP_BLOCKS, SYNTH_DEDUP_FILES])
def test_piece_bytes_equal_the_file_stream(mode):
    offs = [0, 3 << 20, (3 << 20) + 5, (6 << 20) + 77]
    full = synthetic_bytes(offs, 0xC5, mode)
    rng = np.random.default_rng(mode)
    for f in range(3):
        a, b = offs[f], offs[f + 1]
        for _ in range(6):
            s = int(rng.integers(0, max(1, b - a)))
            n = int(rng.integers(0, b - a - s + 1))
            assert np.array_equal(synthetic_piece_bytes(f, s, n, 0xC5, mode), full[a + s:a + s + n])


def _index_for(a, world, params, corrupt=None):
    """The index a GPU run would gather, made by the oracle (file = the piece's global id)."""
    parts = []
    for r in range(world):
        w = workload(a, world, r)
        data = np.concatenate([synthetic_piece_bytes(int(w.ids[i]), int(w.starts[i]),
                                                     w.sizes[i], w.seed, w.mode)
                               for i in range(len(w.sizes))])
        segs, _ = coracle.segment_files(data, w.offs, params, nthreads=8)
        segs["file"] = w.gid[segs["file"]].astype(np.uint32)
        parts.append(segs)
    idx = np.concatenate(parts)
    if corrupt is not None:
        idx["hash"][corrupt, 0] ^= 1
    return idx


def test_sample_parity_passes_and_catches_a_wrong_record():
    p = Ch.Params(average_bits=16, seed=1, min=100_000, max=900_000)
    cp = ChunkParams(p.average_bits, p.seed, p.min, p.max)
    a = _args()
    w0 = workload(a, 3, 0)
    idx = _index_for(a, 3, p)
    r = parity.sample_parity(a, 3, idx, w0.seed, w0.mode, cp, threads=4)
    assert r["gpu_equals_cpu_oracle"] and r["pieces"] == 6 and r["segments"] > 6
    # the last file of rank 1 (gid 15): its first record
    bad = int(np.nonzero(idx["file"] == 15)[0][0])
    r = parity.sample_parity(a, 3, _index_for(a, 3, p, corrupt=bad), w0.seed, w0.mode, cp,
                             threads=4)
    assert not r["gpu_equals_cpu_oracle"] and r["mismatched_pieces"] == [15]


def test_stream_rule_check():
    p = Ch.Params(average_bits=14, seed=1, min=20_000, max=60_000)
    cp = ChunkParams(p.average_bits, p.seed, p.min, p.max)
    n = 3_000_000
    data = synthetic_bytes([0, n], 0xC3)
    segs, _ = coracle.segment_files(data, [0, n], p)
    h = lambda b: hashlib.blake2b(b, digest_size=32).digest()  # noqa: E731
    cand = lambda b: coracle.candidates(b, p)  # noqa: E731
    forced = 0
    for s in segs:
        a, z = int(s["offset"]), int(s["size"])
        assert parity.rule_check(s, data[a:a + z], a, n, cp, cand, h)
        forced += z == p.max
    assert forced > 0 and len(segs) > 40
    s = segs[5].copy()
    s["size"] -= 1  # a cut one byte early
    a = int(s["offset"])
    assert not parity.rule_check(s, data[a:a + int(s["size"])], a, n, cp, cand,
                                 lambda b: bytes(s["hash"]))
