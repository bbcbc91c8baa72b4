"""GPU parity of the re-chunk paths (§8(f) row 4): chunk.Writer.Copy (writer.go:315-420: cheap
copies of whole chunks at chunk boundaries, re-rolled bytes otherwise, read back through
chunk.Get from the store the first writer uploaded to) and MergeFileReader.Hash
(fileset/merge.go:125-143), against the restated Writer in oracle/chunker.py.

The reference's own TestStableHash (fileset/fileset_test.go:202-261) is restated: a file
written by 1, 2, 3 or 7 writers hashes the same through MergeFileReader.Hash as the single
writer's hashDataRefs, on the GPU and in the oracle.
"""
import copy

import numpy as np
import pytest

from conftest import fuzz_cases

from oracle import chunker as Ch
from pfs_amd import _lib
from pfs_amd import chunk as pc
from pfs_amd.cdc import ChunkParams, synthetic_bytes

pytestmark = pytest.mark.gpu

P = Ch.Params(average_bits=10, seed=1, min=500, max=6000)
CP = ChunkParams(P.average_bits, P.seed, P.min, P.max)


def _key(a):
    d = a.next_data_ref
    if d is None:
        return (a.data, None)
    return (a.data, (d.ref.id, d.ref.dek, d.ref.size_bytes, bool(d.ref.edge), d.hash,
                     d.offset_bytes, d.size_bytes))


def gpu_write(parts, store, batch_bytes=1 << 30):
    got, per_file = [], {}
    st = pc.Storage(0, batch_bytes, store=store)

    def cb(anns):
        got.append([_key(a) for a in anns])
        for a in anns:
            if a.next_data_ref is not None:
                per_file.setdefault(a.data, []).append(a.next_data_ref)
    w = st.new_writer("w", cb, pc.with_rolling_hash_config(P.average_bits, P.seed),
                      pc.with_min_max(P.min, P.max))
    for i, part in enumerate(parts):
        w.annotate(pc.Annotation(data=i))
        w.write(part)
    w.close()
    return got, per_file


def oracle_write(parts, store):
    got, per_file = [], {}

    def cb(anns):
        got.append([_key(a) for a in anns])
        for a in anns:
            if a.next_data_ref is not None:
                per_file.setdefault(a.data, []).append(a.next_data_ref)
    w = Ch.Writer(cb=cb, params=P, store=store)
    for i, part in enumerate(parts):
        w.annotate(Ch.Annotation(data=i))
        w.write(part)
    w.close()
    return got, per_file


def as_oracle_refs(refs):
    return [Ch.DataRef(ref=Ch.Ref(size_bytes=d.ref.size_bytes, edge=d.ref.edge, id=d.ref.id,
                                  dek=d.ref.dek), hash=d.hash, offset_bytes=d.offset_bytes,
                       size_bytes=d.size_bytes) for d in refs]


def parts_of(seed, sizes):
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    data = synthetic_bytes(offs, seed).tobytes()
    return [data[int(offs[i]):int(offs[i + 1])] for i in range(len(sizes))], data


def test_first_writer_uploads_and_matches_oracle():
    parts, _ = parts_of(3, [40_000, 700, 0, 25_000, 9_000])
    store = pc.ChunkStore()
    got, _ = gpu_write(parts, store)
    ostore = {}
    want, _ = oracle_write(parts, ostore)
    assert got == want
    assert len(store) == len(ostore)
    for rid, ct in ostore.items():
        assert store.get(rid) == ct  # the uploaded ciphertext (chunk.Create's buf)


@pytest.mark.parametrize("batch_bytes", [1 << 30, 3_000])
def test_copy_stream_matches_oracle(batch_bytes):
    # writer 1 stores files; writer 2 (fileset.Writer.Copy shape: one annotation per file,
    # then Copy of its DataRefs) copies them, interleaved with written files
    parts, _ = parts_of(5, [30_000, 12_000, 800, 45_000, 5_000, 20_000])
    store = pc.ChunkStore()
    _, per_file = gpu_write(parts, store)
    ostore = {}
    _, oper_file = oracle_write(parts, ostore)
    extra, _ = parts_of(6, [7_000, 16_000])
    plan = [("copy", 3), ("write", 0), ("copy", 0), ("copy", 1), ("copy", 5), ("write", 1),
            ("copy", 2), ("copy", 4)]

    got = []
    st = pc.Storage(0, batch_bytes, store=store)
    w = st.new_writer("w2", lambda anns: got.append([_key(a) for a in anns]),
                      pc.with_rolling_hash_config(P.average_bits, P.seed),
                      pc.with_min_max(P.min, P.max))
    want = []
    ow = Ch.Writer(cb=lambda anns: want.append([_key(a) for a in anns]), params=P, store=ostore)
    for k, (op, i) in enumerate(plan):
        w.annotate(pc.Annotation(data=k))
        ow.annotate(Ch.Annotation(data=k))
        if op == "write":
            w.write(extra[i])
            ow.write(extra[i])
        else:
            for d in per_file.get(i, []):
                w.copy(d)
            for d in copy.deepcopy(oper_file.get(i, [])):
                ow.copy(d)
    w.close()
    ow.close()
    assert got == want
    assert w.chunk_count() == ow.chunk_count
    assert w.annotation_count() == ow.annotation_count
    assert len(got) > w.chunk_count(), "no cheap copy (a callback without a new chunk)"


def test_stable_hash_across_writers():
    # fileset_test.go TestStableHash, restated: 1 writer vs 2, 3 and 7 writers
    data = synthetic_bytes([0, 150_000], 8).tobytes()
    store = pc.ChunkStore()
    _, pf = gpu_write([data], store)
    single = pc.hash_data_refs([d.hash for d in pf[0]], params=CP)
    assert single == Ch.file_hash([d.hash for d in pf[0]])
    assert pc.merge_file_hash(store, pf[0], params=CP) == single
    for k in (2, 3, 7):
        size = len(data) // k
        refs, orefs, ostore = [], [], {}
        for off in range(0, len(data), size):
            _, p = gpu_write([data[off:off + size]], store)
            refs += p.get(0, [])
            _, op = oracle_write([data[off:off + size]], ostore)
            orefs += op.get(0, [])
        got = pc.merge_file_hash(store, refs, params=CP)
        want = Ch.merge_file_hash(ostore, copy.deepcopy(orefs), P)
        assert want == single, k
        assert got == single, k


def test_copy_of_tampered_chunk_fails_verification():
    parts, _ = parts_of(9, [20_000])
    store = pc.ChunkStore()
    _, pf = gpu_write(parts, store)
    d = pf[0][0]
    ct = bytearray(store.get(d.ref.id))
    ct[5] ^= 1
    bad = pc.ChunkStore()
    bad.put(d.ref.id, bytes(ct))
    st = pc.Storage(0, store=bad)
    w = st.new_writer("w", None, pc.with_rolling_hash_config(P.average_bits, P.seed),
                      pc.with_min_max(P.min, P.max), pc.with_no_upload())
    w.annotate(pc.Annotation(data=0))
    with pytest.raises(_lib.PfsCdcError) as e:
        w.copy(d)  # the first chunk is an edge chunk: read back (chunk.Get verifyData)
        w.close()
    assert e.value.code == -7


@pytest.mark.parametrize("case", fuzz_cases(6))
def test_copy_random_plans_match_oracle(case):
    """Randomised Copy streams: stored files of random sizes (empty included), a random plan
    of copies (any order, repeats) and written files, a random writer batch size; every
    callback equal to the restated Writer.Copy's."""
    _copy_case(case)


@pytest.mark.parametrize("case", [13, 23, 32, 43, 51, 55, 58])
def test_copy_after_carry_only_probe_flush(case):
    """Regression (round 5, found by the randomised plans): Copy's buf.Len() probe flush
    replayed no bytes of the buffer, only the carried open chunk, which an Annotate cut into a
    chunk (buf.Len() >= avg); whole-chunk copies followed, then written bytes.  The next flush
    took the zero replay count for 'no deferred flush' and re-based the open chunk onto the
    carry, so the following new chunk's Ref.Id (and upload) covered the wrong bytes (its dek
    and DataRef hash were right).  These seeds hit it."""
    _copy_case(case)


def _copy_case(case):
    rng = np.random.default_rng(6600 + case)
    sizes = [0 if rng.random() < 0.1 else int(rng.integers(1, 60_000))
             for _ in range(int(rng.integers(2, 12)))]
    parts, _ = parts_of(20 + case, sizes)
    store = pc.ChunkStore()
    _, per_file = gpu_write(parts, store)
    ostore = {}
    _, oper_file = oracle_write(parts, ostore)
    extra, _ = parts_of(40 + case, [int(rng.integers(0, 30_000)) for _ in range(4)])
    plan = [("copy", int(rng.integers(0, len(parts)))) if rng.random() < 0.7 else
            ("write", int(rng.integers(0, len(extra)))) for _ in range(int(rng.integers(3, 16)))]
    batch = int(rng.choice([1 << 30, 2_500, 20_000]))
    got, want = [], []
    st = pc.Storage(0, batch, store=store)
    w = st.new_writer("w2", lambda anns: got.append([_key(a) for a in anns]),
                      pc.with_rolling_hash_config(P.average_bits, P.seed),
                      pc.with_min_max(P.min, P.max))
    ow = Ch.Writer(cb=lambda anns: want.append([_key(a) for a in anns]), params=P, store=ostore)
    for k, (op, i) in enumerate(plan):
        w.annotate(pc.Annotation(data=k))
        ow.annotate(Ch.Annotation(data=k))
        if op == "write":
            w.write(extra[i])
            ow.write(extra[i])
        else:
            for d in per_file.get(i, []):
                w.copy(d)
            for d in copy.deepcopy(oper_file.get(i, [])):
                ow.copy(d)
    w.close()
    ow.close()
    assert got == want
    assert w.chunk_count() == ow.chunk_count


@pytest.mark.parametrize("case", fuzz_cases(4))
def test_stable_hash_random_splits(case):
    """TestStableHash with random uneven split points: the merged hash of the pieces' DataRefs
    equals the single writer's, on the GPU and in the oracle."""
    rng = np.random.default_rng(7700 + case)
    n = int(rng.integers(20_000, 300_000))
    data = synthetic_bytes([0, n], 30 + case).tobytes()
    store = pc.ChunkStore()
    _, pf = gpu_write([data], store)
    single = pc.hash_data_refs([d.hash for d in pf[0]], params=CP)
    cuts = sorted(set(int(x) for x in rng.integers(1, n, int(rng.integers(1, 9)))))
    bounds = [0] + cuts + [n]
    refs, orefs, ostore = [], [], {}
    for a, b in zip(bounds[:-1], bounds[1:]):
        _, p = gpu_write([data[a:b]], store)
        refs += p.get(0, [])
        _, op = oracle_write([data[a:b]], ostore)
        orefs += op.get(0, [])
    assert Ch.merge_file_hash(ostore, copy.deepcopy(orefs), P) == single
    assert pc.merge_file_hash(store, refs, params=CP) == single
