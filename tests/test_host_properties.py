"""Property tests (hypothesis) of the host-side layout logic every multi-GPU line rests on.
No GPU, no collectives: each function is checked against the invariants its caller needs.

* shard_files / shard_filesets: contiguous ranges that cover every file once, in order, each
  rank within one file of its equal-byte share (the greedy prefix split).
* split_stream: contiguous byte ranges of one stream, borders on the alignment.
* commit_layout: UnorderedWriter.Put's serialization (unordered_writer.go:45-72): each file's
  pieces tile it, every fileset but the last holds exactly memThreshold bytes, and a piece is
  an append exactly when it continues a file.
* select_cuts: Writer.roll's serial rule (writer.go:163-189) over arbitrary candidates.
* encode/decode_primitive: the gathered fileset record round-trips.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from pfs_amd import _lib
from pfs_amd import distributed as pd

SETTINGS = settings(max_examples=150, deadline=None, suppress_health_check=list(HealthCheck))

sizes_st = st.lists(st.integers(0, 5000), min_size=0, max_size=40)


def _check_ranges(ranges, n, world):
    assert len(ranges) == world
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    for (a, b), (c, _) in zip(ranges, ranges[1:]):
        assert a <= b == c


@SETTINGS
@given(sizes=sizes_st, world=st.integers(1, 9))
def test_shard_files_cover_in_order_and_balance(sizes, world):
    ranges = pd.shard_files(sizes, world)
    _check_ranges(ranges, len(sizes), world)
    total, biggest = sum(sizes), max(sizes, default=0)
    for r, (a, b) in enumerate(ranges):
        # rank r's range starts at the first file whose prefix reaches r/world of the bytes,
        # so its bytes differ from the share by less than one file
        assert abs(sum(sizes[a:b]) - total / world) <= biggest + 1


@SETTINGS
@given(n=st.integers(0, 1 << 40), world=st.integers(1, 16),
       align=st.sampled_from([1, 64, 4096]))
def test_split_stream_contiguous_and_aligned(n, world, align):
    ranges = pd.split_stream(n, world, align)
    _check_ranges(ranges, n, world)
    for a, b in ranges[1:]:
        assert a % align == 0 or a == n
    for a, b in ranges:
        assert b - a <= -(-n // world) + align


@SETTINGS
@given(sizes=sizes_st, thr=st.integers(1, 9000))
def test_commit_layout_serializes_like_put(sizes, thr):
    lay = pd.commit_layout(sizes, thr)
    files, starts = lay.file.astype(np.int64), lay.start.astype(np.int64)
    psz = lay.size.astype(np.int64)
    assert list(np.unique(files)) == list(range(len(sizes)))
    assert np.all(np.diff(files) >= 0)
    for f, n in enumerate(sizes):
        idx = np.flatnonzero(files == f)
        # the pieces of a file tile it in order
        assert list(starts[idx]) == list(np.concatenate([[0], np.cumsum(psz[idx])[:-1]]))
        assert int(psz[idx].sum()) == n
    # a piece is an append exactly when it continues its file (the re-Add after a serialize)
    assert list(lay.append) == list(starts > 0)
    fb = lay.fileset_bytes()
    assert int(fb.sum()) == sum(sizes)
    assert np.all(fb[:-1] == thr) and (len(fb) == 0 or fb[-1] <= thr)
    # a continuation always opens a fileset, and a fileset's first piece is either a new file
    # or the continuation of the previous fileset's last file
    begins = set(int(x) for x in lay.fileset_begin[:-1])
    for i in np.flatnonzero(lay.append):
        assert int(i) in begins
    # filesets shard into contiguous piece ranges covering the commit
    for world in (1, 2, 3, 8):
        fs = pd.shard_filesets(lay, world)
        _check_ranges(fs, lay.nfilesets, world)
        pieces = [pd.rank_pieces(lay, r) for r in fs]
        _check_ranges(pieces, lay.npieces, world)


@SETTINGS
@given(n=st.integers(0, 20_000), mn=st.integers(1, 900), extra=st.integers(0, 3000),
       cands=st.lists(st.integers(0, 20_000), max_size=60))
def test_select_cuts_follows_the_roll_rule(n, mn, extra, cands):
    mx = mn + extra
    cs = np.unique(np.asarray([c for c in cands if c < n], dtype=np.uint64))
    offs, sizes, flags = pd.select_cuts(cs, n, mn, mx)
    offs, sizes = offs.astype(np.int64), sizes.astype(np.int64)
    # the segments tile the stream
    assert int(sizes.sum()) == n and (len(offs) == 0 or offs[0] == 0)
    assert np.all(offs[1:] == (offs + sizes)[:-1])
    cset = set(int(c) for c in cs)
    for k, (s, z, f) in enumerate(zip(offs, sizes, flags)):
        assert f & _lib.SEG_VALID
        if f & _lib.SEG_CUT:
            end = int(s + z - 1)
            assert mn <= z <= mx
            # the first candidate at or after s + min - 1, or the forced cut at s + max - 1
            assert end in cset or z == mx
            assert not any(s + mn - 1 <= c < end for c in cset)
        else:  # the open tail: the last segment, which would not reach a cut
            assert k == len(offs) - 1
            assert not any(s + mn - 1 <= c < n for c in cset) and z < mx


@SETTINGS
@given(add=st.one_of(st.none(), st.binary(max_size=300)),
       dele=st.one_of(st.none(), st.binary(max_size=300)),
       size=st.integers(-(1 << 63), (1 << 63) - 1))
def test_primitive_record_roundtrips(add, dele, size):
    assert pd.decode_primitive(pd.encode_primitive(add, dele, size)) == (add, dele, size)


@pytest.mark.parametrize("world", [1, 2, 5])
def test_pack_index_roundtrip_random(world):
    rng = np.random.default_rng(world)
    dt = _lib.segment_dtype()
    cap, blocks, want = 17, [], []
    for r in range(world):
        n = int(rng.integers(0, cap + 1))
        seg = np.zeros(n, dtype=dt)
        for name in dt.names:
            if seg[name].dtype.kind == "u" and seg[name].ndim == 1:
                seg[name] = rng.integers(0, 1 << 30, n)
        blocks.append(pd.pack_index(seg, 1000 * r, cap))
        w = seg.copy()
        w["file"] = w["file"] + 1000 * r
        want.append(w)
    got = pd.unpack_index(np.concatenate(blocks), world, cap)
    assert got.tobytes() == np.concatenate(want).tobytes()
