"""GPU tests of the device group (pfscdc_group_*, pfscdc_uw_create_group): one process, several
contexts, the work of one call dealt across them and the chunk-ref index gathered peer to peer
onto the index device.  On the one-GPU box every member is device 0, so N = 2/4/8 members are
N contexts sharing the GPU: the same dealing, concurrent member scans and gather code as N
devices.  Done-when: records, per-file ranges, Refs, the unordered
writer's ordered event stream, every fileset root and the index digest bit-identical to one
ctx; the one-ctx results are themselves checked against the oracle here and in
test_gpu_parity.py / test_gpu_fileset.py.
"""
import hashlib

import numpy as np
import pytest

from conftest import fuzz_cases

from oracle import chunker as Ch
from oracle import coracle
from oracle import fileset as OF
from pfs_amd import _lib
from pfs_amd import fileset as PF
from pfs_amd.cdc import ChunkParams, Chunker, synthetic_bytes
from pfs_amd.group import DeviceGroup, deal

pytestmark = pytest.mark.gpu

SMALL = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
SMALL_INDEX = Ch.Params(average_bits=13, seed=0, min=3000, max=60000)


def cp(p):
    return ChunkParams(p.average_bits, p.seed, p.min, p.max)


def same_result(a, b):
    assert np.array_equal(a.file_begin, b.file_begin)
    assert a.segments.tobytes() == b.segments.tobytes()
    if a.refs is not None or b.refs is not None:
        assert a.refs.tobytes() == b.refs.tobytes()


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("case", fuzz_cases(2))
def test_group_scan_host_equals_one_ctx_and_oracle(n, case):
    rng = np.random.default_rng(7100 + 10 * n + case)
    p = [SMALL, Ch.Params(average_bits=10, seed=2, min=64, max=5000)][case % 2]
    nf = int(rng.integers(1, 90))
    lens = rng.integers(0, 5 * p.max, nf)
    lens[rng.random(nf) < 0.2] = 0
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 40 + case)
    one = Chunker(cp(p), 0, ref_ids=True)
    g = DeviceGroup([0] * n, cp(p), ref_ids=True)
    want = one.scan(data, offs)
    got = g.scan(data, offs)
    same_result(want, got)
    assert np.array_equal(g.part_begin(), deal(offs, n))
    segs, begin = coracle.segment_files(data, offs, p, nthreads=4)
    assert np.array_equal(got.file_begin, begin)
    for k in ("offset", "size", "file", "flags", "hash"):
        assert np.array_equal(got.segments[k], segs[k]), k
    t = g.timings()
    assert t["gather_bytes"] == len(got.segments) * (56 + 64)
    sp, rp, dev = g.index_device()
    assert dev == 0 and (sp != 0) == (len(got.segments) > 0)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_group_scan_resident_reference_params(n):
    """configs[1]-shaped: many 4 MiB-ish files generated in place on the members, the
    reference chunking parameters; equal to one ctx over the same bytes."""
    import torch

    rng = np.random.default_rng(900 + n)
    lens = rng.integers(1, 3 * (4 << 20), 48)
    lens[5] = 0
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    g = DeviceGroup([0] * n, ChunkParams(), ref_ids=True)
    parts = g.fill_synthetic_resident(offs, 0xC2)
    got = g.scan_resident(parts, offs)
    one = Chunker(ChunkParams(), 0, ref_ids=True)
    dev = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
    one.fill_synthetic(dev, offs, 0xC2)
    want = one.scan(dev, offs)
    same_result(want, got)
    # a caller-chosen dealing (uneven, with empty members) gives the same records
    pb = np.array(sorted(rng.integers(0, 49, n - 1).tolist()), dtype=np.uint32)
    pb = np.concatenate([[0], pb, [48]]).astype(np.uint32)
    # (each member its own allocation: a member's bytes must start 16-byte aligned)
    parts = [dev[int(offs[pb[k]]):int(offs[pb[k + 1]])].clone() for k in range(n)]
    same_result(want, g.scan_resident(parts, offs, pb))
    assert np.array_equal(g.part_begin(), pb)


def test_group_scan_errors():
    g = DeviceGroup([0, 0], cp(SMALL))
    offs = np.array([0, 100, 200], dtype=np.uint64)
    with pytest.raises(_lib.PfsCdcError) as e:
        g.scan_resident([None, None], offs)  # members with bytes but no buffer
    assert e.value.code == _lib.PFSCDC_EINVAL
    with pytest.raises(_lib.PfsCdcError):
        g.scan_resident([None, None], offs, [0, 3, 2])  # part_begin not monotone
    with pytest.raises(_lib.PfsCdcError):
        DeviceGroup([0, 99], cp(SMALL))  # no such device
    r = g.scan(np.zeros(0, dtype=np.uint8), [0])  # no files
    assert len(r.segments) == 0 and list(r.file_begin) == [0]


def uw_run(storage, ops):
    w = storage.new_unordered_writer()
    for op in ops:
        if op[0] == "put":
            w.put(*op[1:])
        else:
            w.delete(*op[1:])
    prims = w.close()
    log = list(w.log)
    w.release()
    return prims, log


def index_digest(prims):
    h = hashlib.blake2b(digest_size=32)
    for p in prims:
        for r in (p.additive, p.deletive):
            h.update(b"\x00" if r is None else b"\x01" + len(r).to_bytes(8, "little") + r)
        h.update(int(p.size_bytes).to_bytes(8, "little"))
    return h.hexdigest()


def workload(seed, nfiles, max_len):
    rng = np.random.default_rng(seed)
    data = synthetic_bytes([0, nfiles * max_len], seed).tobytes()
    ops, pos = [], 0
    for i in range(nfiles):
        ln = 0 if i % 11 == 0 else int(rng.integers(1, max_len))
        path = f"/d{int(rng.integers(0, 4))}/f{int(rng.integers(0, nfiles)):05d}"
        ops.append(("put", path, ["", "t1"][int(rng.integers(0, 2))], bool(rng.integers(0, 4) == 0),
                    data[pos:pos + ln]))
        pos += ln
        if i % 17 == 16:
            ops.append(("delete", ops[-2][1], ""))
    return ops


@pytest.mark.parametrize("n", [2, 4, 8])
def test_group_unordered_writer_equals_one_ctx(n, knob):
    """Serialized filesets dealt round robin over n members: the ordered event stream (every
    chunk of every data and index stream with its Ref.Id, every level-0 index entry), every
    fileset's roots and the index digest equal one ctx writing the same groups, and the
    restated reference."""
    ops = workload(50 + n, 400, 40_000)
    inflight = 600_000
    knob("PFSCDC_UW_INFLIGHT", inflight)
    one = PF.Storage(0, cp(SMALL), 300_000, cp(SMALL_INDEX))
    want, wlog = uw_run(one, ops)
    knob("PFSCDC_UW_INFLIGHT", inflight * n)  # n members share the writer's in-flight bytes
    grp = PF.Storage(0, cp(SMALL), 300_000, cp(SMALL_INDEX), devices=[0] * n)
    got, glog = uw_run(grp, ops)
    assert len(want) >= 2 * n, "too few filesets to reach every member"
    assert glog == wlog
    assert got == want
    assert index_digest(got) == index_digest(want)
    # and the reference restatement, fileset by fileset
    ow = OF.UnorderedWriter(SMALL, 300_000, SMALL_INDEX)
    for op in ops:
        (ow.put if op[0] == "put" else ow.delete)(*op[1:])
    ref = ow.close()
    assert [(p.additive, p.deletive, p.size_bytes) for p in got] == \
        [(r.additive, r.deletive, r.size_bytes) for r in ref]


@pytest.mark.parametrize("mirror", ["1", "0"])
def test_group_unordered_writer_reference_params_and_reuse(mirror, knob):
    """Reference chunking, Puts above the copy pool's split, a file cut across filesets, more
    members than groups at first; the Storage reuses its group for a second writer."""
    knob("PFSCDC_UW_MIRROR", mirror)
    knob("PFSCDC_UW_INFLIGHT", 40_000_000)
    data = synthetic_bytes([0, 50 << 20], 21).tobytes()
    ops = [("put", f"/f{i}", "", False, data[i * (9 << 20):(i + 1) * (9 << 20)]) for i in range(5)]
    ops.append(("put", "/g", "", False, data[45 << 20:]))
    one = PF.Storage(0, ChunkParams(), 10_000_000)
    want, wlog = uw_run(one, ops)
    grp = PF.Storage(0, ChunkParams(), 10_000_000, devices=[0, 0, 0])
    for _ in range(2):
        got, glog = uw_run(grp, ops)
        assert got == want
        # per-stream equality (the grouping differs from one ctx's 40 MB groups)
        for fs in range(len(want)):
            assert [e for e in glog if e[0] == fs and e[1] == "chunk" and e[2] == -1] == \
                [e for e in wlog if e[0] == fs and e[1] == "chunk" and e[2] == -1]


def test_ordered_events_with_two_group_writers(knob):
    """PFSCDC_UW_WORKERS = 2 on one device now emits group by group: the whole event stream
    equals one group writer's."""
    ops = workload(77, 160, 40_000)
    knob("PFSCDC_UW_INFLIGHT", 500_000)
    st = PF.Storage(0, cp(SMALL), 250_000, cp(SMALL_INDEX))
    want, wlog = uw_run(st, ops)
    knob("PFSCDC_UW_WORKERS", 2)
    st2 = PF.Storage(0, cp(SMALL), 250_000, cp(SMALL_INDEX))
    got, glog = uw_run(st2, ops)
    assert got == want and glog == wlog


@pytest.mark.parametrize("case", fuzz_cases(6))
def test_group_unordered_writer_random_ops_equal_one_ctx(case, knob):
    """Random Put/Delete sequences (memThreshold splits, exact fills, appends, overwrites,
    tags, file and directory deletes) over a device group of 1-8 ctxs, with the writer's own
    forms drawn per case: the ordered event stream equals one ctx writing the same groups,
    and the filesets equal the restated reference."""
    from test_gpu_fileset import RAND_INDEX, random_ops

    rng = np.random.default_rng(7700 + case)
    n = int(rng.integers(1, 9))
    thr = int(rng.integers(60_000, 400_000))
    group = int(rng.choice([thr, 2 * thr, 3 * thr + 1]))
    knob("PFSCDC_UW_MIRROR", int(rng.integers(0, 2)))
    knob("PFSCDC_UW_INDEX_GROUPED", int(rng.integers(0, 2)))
    data = synthetic_bytes([0, 8 << 20], 170 + case).tobytes()
    paths = [f"/d{int(rng.integers(0, 3))}/s{int(rng.integers(0, 2))}/f{j:03d}"
             for j in range(int(rng.integers(3, 40)))]
    ops = random_ops(rng, data, int(rng.integers(40, 200)), paths, thr)
    knob("PFSCDC_UW_INFLIGHT", group)
    want, wlog = uw_run(PF.Storage(0, cp(SMALL), thr, cp(RAND_INDEX)), ops)
    knob("PFSCDC_UW_INFLIGHT", group * n)
    got, glog = uw_run(PF.Storage(0, cp(SMALL), thr, cp(RAND_INDEX), devices=[0] * n), ops)
    assert glog == wlog
    assert got == want
    ow = OF.UnorderedWriter(SMALL, thr, RAND_INDEX)
    for op in ops:
        (ow.put if op[0] == "put" else ow.delete)(*op[1:])
    ref = ow.close()
    assert [(p.additive, p.deletive, p.size_bytes) for p in got] == \
        [(r.additive, r.deletive, r.size_bytes) for r in ref]


@pytest.mark.parametrize("case", fuzz_cases(4))
def test_group_scan_resident_random_dealing_equal_one_ctx(case):
    """Caller-chosen dealings (empty members, one member holding everything, uneven splits)
    over 1-8 ctxs, with Ref ids on or off, equal one ctx over the same bytes."""
    import torch

    rng = np.random.default_rng(7900 + case)
    n = int(rng.integers(1, 9))
    p = [SMALL, Ch.Params(average_bits=14, seed=3, min=4000, max=90000)][case % 2]
    nf = int(rng.integers(0, 120))
    lens = rng.integers(0, 6 * p.max, nf)
    lens[rng.random(nf) < 0.2] = 0
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    ref_ids = bool(rng.integers(0, 2))
    one = Chunker(cp(p), 0, ref_ids=ref_ids)
    dev = torch.empty(max(int(offs[-1]), 1), dtype=torch.uint8, device="cuda:0")
    one.fill_synthetic(dev, offs, 300 + case)
    want = one.scan(dev[:int(offs[-1])], offs)
    g = DeviceGroup([0] * n, cp(p), ref_ids=ref_ids)
    pb = np.concatenate([[0], np.sort(rng.integers(0, nf + 1, n - 1)), [nf]]).astype(np.uint32)
    parts = [dev[int(offs[pb[k]]):int(offs[pb[k + 1]])].clone() if pb[k + 1] > pb[k] else None
             for k in range(n)]
    got = g.scan_resident(parts, offs, pb)
    same_result(want, got)


@pytest.mark.parametrize("case", fuzz_cases(6))
def test_group_scan_stream_equals_one_ctx(case):
    """One stream split across 1-8 ctxs (equal byte ranges, the 64-byte window in front, the
    serial selection over the gathered candidates, each segment hashed by the member holding
    its first byte) equals one ctx's scan of the stream: random bytes, dense candidates, and a
    run of zeros whose forced max-size cuts straddle the members' borders."""
    rng = np.random.default_rng(8100 + case)
    n = int(rng.integers(1, 9))
    p = [SMALL, Ch.Params(average_bits=8, seed=2, min=64, max=3000),
         Ch.Params(average_bits=14, seed=1, min=5000, max=40000)][case % 3]
    nb = int(rng.integers(0, 3 << 20)) if case % 4 else int(rng.integers(0, 200))
    data = synthetic_bytes([0, nb], 500 + case)
    if case % 2 and nb > 1000:
        a = int(rng.integers(0, nb // 2))
        data[a:a + int(rng.integers(1, nb - a))] = 0  # forced cuts at max inside the zero run
    one = Chunker(cp(p), 0)
    want = one.scan(data, [0, nb])
    g = DeviceGroup([0] * n, cp(p))
    got = g.scan_stream(data)
    same_result(want, got)
    assert g.part_begin() is None


def test_group_scan_stream_reference_params():
    """configs[2]'s shape at 64 MiB: the reference chunking, four ctxs, forced 20 MB cuts."""
    data = synthetic_bytes([0, 64 << 20], 0xC3)
    data[20 << 20:50 << 20] = 7  # a constant run: forced cuts at 20 MB
    one = Chunker(ChunkParams(), 0)
    want = one.scan(data, [0, len(data)])
    got = DeviceGroup([0, 0, 0, 0], ChunkParams()).scan_stream(data)
    same_result(want, got)
    assert any(int(s) == 20_000_000 for s in got.segments["size"])
