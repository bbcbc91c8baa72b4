"""GPU parity of pachd-level stream formation (§8(f) rows 2-3): UnorderedWriter -> fileset.Writer
-> chunk.Writer (GPU) -> multilevel index.Writer, against the restated reference
(oracle/fileset.py over oracle/chunker.py).

Compared per serialized fileset: SizeBytes, the encoded root index.Index of the additive and
deletive indexes (which pins, through Range.ChunkRef, every index chunk's Ref.Id and so every
entry and every data chunk Ref beneath it), every level-0 index entry (pbutil frame) and the
chunk sequence of every stream (size, edge, Ref.Id).  Workloads cover memThreshold splits
(including a Put that ends exactly at the threshold, which leaves an empty entry in the next
fileset), appends, overwrites, tags, empty files, file and directory deletes, and a multilevel
index (small index chunking params as a test hook; the reference's own 20-bit index chunking
is run as well).
"""
import numpy as np
import pytest

from conftest import fuzz_cases

from oracle import chunker as Ch
from oracle import fileset as OF
from pfs_amd import _lib
from pfs_amd import fileset as PF
from pfs_amd.cdc import ChunkParams, synthetic_bytes

pytestmark = pytest.mark.gpu

SMALL = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
# index chunking test hook: small enough for several levels, with avg above the largest entry
# (an entry >= avg is cut before at every level, so levels would never converge; the
# reference's 1 MiB avg rules that out)
SMALL_INDEX = Ch.Params(average_bits=13, seed=0, min=3000, max=60000)


def cp(p):
    return ChunkParams(p.average_bits, p.seed, p.min, p.max)


def streams(log):
    """Per stream: chunk (size, edge, id) sequences and index-entry sequences."""
    out = {}
    for e in log:
        if e[0] == "chunk":
            out.setdefault(("chunk", e[1], e[2]), []).append(e[3:])
        else:
            out.setdefault(("index", e[1]), []).append(e[2])
    return out


def run_both(ops, p, mem_threshold, index_params=None):
    ow = OF.UnorderedWriter(p, mem_threshold, index_params)
    st = PF.Storage(0, cp(p), mem_threshold, cp(index_params) if index_params else None)
    pw = st.new_unordered_writer()
    for op in ops:
        if op[0] == "put":
            ow.put(*op[1:])
            pw.put(*op[1:])
        else:
            ow.delete(*op[1:])
            pw.delete(*op[1:])
    want = ow.close()
    got = pw.close()
    return want, got, ow.log, pw.events


def check(want, got, wlog, glog):
    assert len(got) == len(want)
    for i, (w, g) in enumerate(zip(want, got)):
        assert g.size_bytes == w.size_bytes, i
        assert (g.num_files, g.num_deletes) == (len(w.files), len(w.deletes)), i
        ws, gs = streams(wlog[i]), streams(glog[i] if i < len(glog) else [])
        assert sorted(gs) == sorted(ws), i
        for k in ws:
            assert gs[k] == ws[k], (i, k)
        assert g.additive == w.additive, i
        assert g.deletive == w.deletive, i


def workload(seed, nfiles, max_len, dirs=4):
    rng = np.random.default_rng(seed)
    data = synthetic_bytes([0, nfiles * max_len], seed).tobytes()
    ops, pos = [], 0
    for i in range(nfiles):
        n = 0 if i % 11 == 0 else int(rng.integers(1, max_len))
        path = f"/d{int(rng.integers(0, dirs))}/f{int(rng.integers(0, nfiles)):05d}"
        tag = ["", "default", "t1", "t2"][int(rng.integers(0, 4))]
        ops.append(("put", path, tag, bool(rng.integers(0, 4) == 0), data[pos:pos + n]))
        pos += n
        if i % 17 == 16:
            ops.append(("delete", ops[-2][1], ""))
    return ops, data


@pytest.mark.parametrize("index_grouped", ["1", "0"])
@pytest.mark.parametrize("inflight", [None, "300000"])
def test_unordered_writer_many_filesets_multilevel_index(inflight, index_grouped, knob):
    # inflight: serialized filesets are written in groups of up to this many bytes (the
    # default holds all of them until Close); the output must not depend on the grouping.
    # index_grouped: a group's index writers closed level by level in grouped closes (the
    # default) or one fileset at a time
    knob("PFSCDC_UW_INDEX_GROUPED", index_grouped)
    if inflight:
        knob("PFSCDC_UW_INFLIGHT", inflight)
    ops, _ = workload(1, 160, 40_000)
    ops.append(("delete", "/d1/", ""))
    ops.append(("put", "/d1/again", "", False, b"xyz" * 1000))
    want, got, wlog, glog = run_both(ops, SMALL, 400_000, SMALL_INDEX)
    assert len(want) >= 5
    assert any(e[0] == "chunk" and e[1] == 0 and e[2] >= 2 for log in wlog for e in log), \
        "no multilevel index"
    check(want, got, wlog, glog)


def test_put_ending_exactly_at_threshold_leaves_empty_entry():
    data = synthetic_bytes([0, 300_000], 7).tobytes()
    ops = [("put", "/a", "", False, data[:100_000]), ("put", "/b", "", False, data[100_000:250_000]),
           ("put", "/c", "", False, data[250_000:300_000])]
    want, got, wlog, glog = run_both(ops, SMALL, 250_000, SMALL_INDEX)
    assert ("/b", "default") in want[1].files  # the empty re-Add of io.CopyN's exact fill
    check(want, got, wlog, glog)


def test_large_file_split_across_filesets_reference_index_params():
    # default data chunking and the reference's own index chunking (avgBits 20, seed = level)
    data = synthetic_bytes([0, 26 << 20], 9).tobytes()
    ops = [("put", f"/f{i}", "", False, data[i * (3 << 20):(i + 1) * (3 << 20)]) for i in range(4)]
    ops.append(("put", "/big", "", False, data[12 << 20:]))
    want, got, wlog, glog = run_both(ops, Ch.Params(), 10_000_000)
    assert len(want) == 3
    check(want, got, wlog, glog)


def test_writer_errors_are_sticky():
    st = PF.Storage(0, cp(SMALL), 100_000, cp(SMALL_INDEX))
    w = st.new_unordered_writer()
    w.put("/x", "", False, b"abc")
    w.close()
    with pytest.raises(_lib.PfsCdcError):
        w.put("/y", "", False, b"abc")


def test_reference_index_params_many_small_files_multilevel():
    # ~6,000 small files: ~1.3 MB of level-0 index entries, so the reference's own index
    # chunking (avgBits 20, 1 MB / 20 MB, seed = level) cuts level 0 and builds level 1
    data = synthetic_bytes([0, 6000 * 97], 13).tobytes()
    ops = [("put", f"/dir{i % 7}/file-{i:06d}", "", False, data[i * 97:(i + 1) * 97])
           for i in range(6000)]
    want, got, wlog, glog = run_both(ops, Ch.Params(), 10 ** 9)
    levels = {e[2] for e in wlog[0] if e[0] == "chunk" and e[1] == 0}
    assert max(levels) >= 1, levels
    check(want, got, wlog, glog)


@pytest.mark.parametrize("workers,mirror", [("2", "1"), ("3", "0"), ("1", "0")])
def test_group_writers_and_upload_paths(workers, mirror, knob):
    """Round-3 write path: several groups in flight on group writers of their own ctxs
    (PFSCDC_UW_WORKERS), Put bytes uploaded into arena device mirrors as they arrive or
    uploaded at group time (PFSCDC_UW_MIRROR), the union hash launch per grouped close: the
    output must equal the restated reference whatever the grouping and upload path."""
    knob("PFSCDC_UW_INFLIGHT", 300000)
    knob("PFSCDC_UW_WORKERS", workers)
    knob("PFSCDC_UW_MIRROR", mirror)
    ops, _ = workload(3, 160, 40_000)
    want, got, wlog, glog = run_both(ops, SMALL, 400_000, SMALL_INDEX)
    assert len(want) >= 5
    check(want, got, wlog, glog)


@pytest.mark.parametrize("workers", ["1", "2"])
def test_large_puts_copy_pool_reference_params(workers, knob):
    """Puts above the copy pool's 4 MiB split (the persistent copy threads) and files split
    across filesets, at the reference's chunking; one and two group writers."""
    knob("PFSCDC_UW_WORKERS", workers)
    knob("PFSCDC_UW_INFLIGHT", 15000000)
    data = synthetic_bytes([0, 40 << 20], 11).tobytes()
    ops = [("put", f"/f{i}", "", False, data[i * (9 << 20):(i + 1) * (9 << 20)]) for i in range(4)]
    ops.append(("put", "/g", "", False, data[36 << 20:]))
    want, got, wlog, glog = run_both(ops, Ch.Params(), 10_000_000)
    assert len(want) == 5
    check(want, got, wlog, glog)


def test_trim_cache_frees_pooled_arenas_and_writers_still_agree():
    """the arenas (page-locked host bytes + device mirrors) and contexts a destroyed
    writer leaves for the next one are freed by Storage.trim / pfscdc_uw_trim_cache, and a
    writer made after a trim allocates afresh and still equals the restated reference."""
    lib = _lib.load()
    ops, _ = workload(5, 60, 40_000)
    st = PF.Storage(0, cp(SMALL), 400_000, cp(SMALL_INDEX))
    pw = st.new_unordered_writer()
    for op in ops:
        (pw.put if op[0] == "put" else pw.delete)(*op[1:])
    pw.close()
    pw.release()
    assert lib.pfscdc_uw_cached_arena_bytes() > 0  # the written filesets' arenas were pooled
    out = st.trim()
    assert out["data_contexts"] >= 1 and out["arena_bytes"] > 0
    assert lib.pfscdc_uw_cached_arena_bytes() == 0
    want, got, wlog, glog = run_both(ops, SMALL, 400_000, SMALL_INDEX)
    check(want, got, wlog, glog)


def random_ops(rng, data, nops, paths, thr):
    """Random Put/delete sequence: appends and overwrites of a small path set (so paths repeat
    across filesets), tags, empty Puts, Puts sized to the threshold, file and directory
    deletes."""
    ops, pos = [], 0
    for _ in range(nops):
        r = rng.random()
        path = paths[int(rng.integers(0, len(paths)))]
        if r < 0.12:
            ops.append(("delete", path, ""))
        elif r < 0.17:
            ops.append(("delete", path[:path.rindex("/") + 1], ""))
        else:
            k = rng.random()
            n = 0 if k < 0.1 else thr if k < 0.15 else thr // 2 if k < 0.2 else \
                int(rng.integers(1, thr // 3))
            n = min(n, len(data) - pos)
            tag = ["", "default", "t1"][int(rng.integers(0, 3))]
            ops.append(("put", path, tag, bool(rng.integers(0, 3) == 0), data[pos:pos + n]))
            pos += n
    return ops


# Index chunking for the randomised workloads: min above the largest possible entry (a file
# piece is at most memThreshold = 400 KB, so at most ~200 DataRefs at SMALL's 2,000-byte min,
# ~20 KB encoded).  An entry at or above the index min can be cut inside the level above a
# level that closed with one annotation in one chunk, i.e. inside a level Close never closes;
# the reference then races that level's callback against Close's return (index/writer.go:100,
# 121-123, 148-161).  With the reference's parameters an entry is at most ~100 KB (1e9-byte
# filesets of >= 1 MB chunks) against a 1 MB index min, so it never happens; DESIGN §5.
RAND_INDEX = Ch.Params(average_bits=16, seed=0, min=40_000, max=400_000)


@pytest.mark.parametrize("case", fuzz_cases(8))
def test_unordered_writer_random_ops_equal_oracle(case, knob):
    """Randomised Put/delete sequences against the restated UnorderedWriter (memThreshold
    splits, exact fills, appends, overwrites, tags, file and directory deletes), with index
    chunking small enough for several levels, and the writer's own forms drawn per case
    (group writers, group size, upload during the Puts, grouped index closes): none may
    change a result."""
    rng = np.random.default_rng(3100 + case)
    thr = int(rng.integers(60_000, 400_000))
    knob("PFSCDC_UW_WORKERS", int(rng.integers(1, 3)))
    knob("PFSCDC_UW_INFLIGHT", int(rng.choice([1 << 35, 3 * thr, 700_000])))
    knob("PFSCDC_UW_MIRROR", int(rng.integers(0, 2)))
    knob("PFSCDC_UW_INDEX_GROUPED", int(rng.integers(0, 2)))
    data = synthetic_bytes([0, 6 << 20], 90 + case).tobytes()
    paths = [f"/d{int(rng.integers(0, 3))}/s{int(rng.integers(0, 2))}/f{j:03d}"
             for j in range(int(rng.integers(3, 40)))]
    ops = random_ops(rng, data, int(rng.integers(20, 160)), paths, thr)
    want, got, wlog, glog = run_both(ops, SMALL, thr, RAND_INDEX)
    check(want, got, wlog, glog)


@pytest.mark.parametrize("case", fuzz_cases(6))
def test_unordered_writer_tricky_paths_equal_oracle(case):
    """Paths and tags that stress the Buffer's byte-wise (path, tag) order and the prefix
    match of directory deletes (buffer.go:70-106, unordered_writer.go): shared prefixes of
    different lengths ('/a', '/a/b', '/ab', '/a-b'), non-ASCII UTF-8, deep nesting, tags
    sorting around '' and 'default', deletes of '/', of a file's own path with a trailing
    slash, and of directories that do not exist."""
    rng = np.random.default_rng(3300 + case)
    atoms = ["a", "b", "ab", "a-b", "a.b", "é", "日本", "z", "A", "0", "a b"]
    paths = []
    for _ in range(int(rng.integers(5, 30))):
        depth = int(rng.integers(1, 5))
        paths.append("/" + "/".join(atoms[int(rng.integers(0, len(atoms)))] for _ in range(depth)))
    tags = ["", "default", "Default", "t", "t0", "é"]
    thr = int(rng.integers(30_000, 200_000))
    data = synthetic_bytes([0, 3 << 20], 130 + case).tobytes()
    ops, pos = [], 0
    for _ in range(int(rng.integers(20, 100))):
        r = rng.random()
        path = paths[int(rng.integers(0, len(paths)))]
        if r < 0.1:
            ops.append(("delete", path, tags[int(rng.integers(0, len(tags)))]))
        elif r < 0.18:
            d = path[:path.rindex("/") + 1] if rng.random() < 0.7 else \
                ["/", path + "/", "/nothing/"][int(rng.integers(0, 3))]
            ops.append(("delete", d, ""))
        else:
            n = min(int(rng.integers(0, thr // 2)), len(data) - pos)
            ops.append(("put", path, tags[int(rng.integers(0, len(tags)))],
                        bool(rng.integers(0, 3) == 0), data[pos:pos + n]))
            pos += n
    want, got, wlog, glog = run_both(ops, SMALL, thr, RAND_INDEX)
    check(want, got, wlog, glog)
