"""CPU-only checks of the oracle against itself and against the reference's own property
tests (restated from /root/reference/src/internal/storage/chunk/chunk_test.go and
fileset/fileset_test.go, which pin properties, not bits — SURVEY.md §4, §8c).

* literal byte-by-byte Writer == numpy closed form == C restatement (segments, digests)
* TestWriteThenRead (chunk_test.go:39-53, sizes :32-37): DataRefs re-read in order
  reproduce every annotation's bytes
* Write segmentation independence: splitting an annotation's bytes over many Write calls
  does not move a cut (roll keeps numChunkBytesAnnotation across calls, writer.go:163-196)
* TestStableHash analogue (fileset_test.go:202-261): FileInfo.Hash of a file is identical
  whatever other files surround it in the stream (hash/seglen reset at Annotate)
"""
import numpy as np
import pytest

from oracle import chunker as Ch
from oracle import coracle
from pfs_amd.cdc import synthetic_bytes

SMALL = Ch.Params(average_bits=10, seed=1, min=500, max=4000)


def files_from(seed, n, max_len):
    rng = np.random.default_rng(seed)
    lens = [int(x) for x in rng.integers(0, max_len, n)]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, seed)
    return [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(n)], data, offs


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_literal_equals_numpy_equals_c(seed):
    files, data, offs = files_from(seed, 25, 9000)
    lit = Ch.chunk_stream(files, SMALL, "literal")
    fast = Ch.chunk_stream(files, SMALL, "numpy")
    assert [(c.data, c.edge) for c in lit] == [(c.data, c.edge) for c in fast]
    fl = Ch.file_segments_from_chunks(lit, len(files))
    assert fl == Ch.file_segments_from_chunks(fast, len(files))
    segs, begin = coracle.segment_files(data, offs, SMALL, nthreads=3)
    for f in range(len(files)):
        got = [(int(s["offset"]), int(s["size"]), bytes(s["hash"]))
               for s in segs[int(begin[f]):int(begin[f + 1])]]
        assert got == fl[f]


def test_literal_segments_default_params_small_file():
    f = synthetic_bytes([0, 70_000], 3).tobytes()
    assert Ch.segments_literal(f, Ch.Params()) == Ch.segments_numpy(f, Ch.Params()) == \
        [(0, 70_000, False)]


@pytest.mark.parametrize("max_ann,total", [(1000, 1000), (1000, 100_000), (50_000, 600_000)])
def test_write_then_read(max_ann, total):
    # chunk_test.go generateAnnotations: sizes rand.Intn(max)+1 until total is used
    rng = np.random.default_rng(max_ann + total)
    sizes, left = [], total
    while left > 0:
        s = min(int(rng.integers(0, max_ann)) + 1, left)
        sizes.append(s)
        left -= s
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    data = synthetic_bytes(offs, 77)
    files = [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(len(sizes))]
    chunks = Ch.chunk_stream(files, SMALL, "numpy")
    store = {c.index: c.data for c in chunks}
    per_file = [[] for _ in files]
    for c in chunks:
        for a in c.annotations:
            if a.next_data_ref is not None:
                per_file[a.data].append(a.next_data_ref)
    for i, f in enumerate(files):
        got = b"".join(store[d.ref.chunk_index][d.offset_bytes:d.offset_bytes + d.size_bytes]
                       for d in per_file[i])
        assert got == f


def test_write_segmentation_independence():
    f = synthetic_bytes([0, 50_000], 5).tobytes()
    w1 = Ch.Writer(params=SMALL)
    w1.annotate(Ch.Annotation(data=0))
    w1.write(f)
    w1.close()
    w2 = Ch.Writer(params=SMALL)
    w2.annotate(Ch.Annotation(data=0))
    rng = np.random.default_rng(1)
    cuts = sorted(int(x) for x in rng.integers(0, len(f), 37))
    prev = 0
    for c in cuts + [len(f)]:
        w2.write(f[prev:c])
        prev = c
    w2.close()
    assert [c.data for c in w1.chunks] == [c.data for c in w2.chunks]


def test_stable_file_hash_independent_of_neighbours():
    files, _, _ = files_from(11, 12, 20_000)
    base = Ch.file_segments_from_chunks(Ch.chunk_stream(files, SMALL), len(files))
    for k in range(1, 4):
        sub = files[k:k + 5]
        other = Ch.file_segments_from_chunks(Ch.chunk_stream(sub, SMALL), len(sub))
        for j in range(len(sub)):
            assert Ch.file_hash([h for _, _, h in other[j]]) == \
                Ch.file_hash([h for _, _, h in base[k + j]])


def test_zero_byte_file_hash_is_blake2b_empty():
    chunks = Ch.chunk_stream([b"", b"abc", b""], SMALL)
    segs = Ch.file_segments_from_chunks(chunks, 3)
    assert segs[0] == [] and segs[2] == []
    assert Ch.file_hash([]).hex().startswith("0e5751c026e543b2")


def test_close_after_cut_emits_empty_last_chunk():
    f = synthetic_bytes([0, 40_000], 8).tobytes()
    segs = Ch.segments_numpy(f, SMALL)
    end = [s for s in segs if s[2]][-1]
    g = f[:end[0] + end[1]]
    chunks = Ch.chunk_stream([g], SMALL, "literal")
    assert chunks[-1].data == b"" and chunks[-1].edge
    assert all(a.next_data_ref is None for a in chunks[-1].annotations)


def test_annotate_cuts_before_file_when_open_chunk_reaches_avg():
    p = Ch.Params(average_bits=12, seed=1, min=3000, max=50_000)
    files = [synthetic_bytes([0, 1500], i).tobytes() for i in range(8)]  # all < min
    chunks = Ch.chunk_stream(files, p, "literal")
    # chunk boundaries fall exactly where the open buffer first reaches >= 4096 at Annotate
    sizes = [len(c.data) for c in chunks]
    assert sizes[:-1] == [4500, 4500] and sum(sizes) == 8 * 1500


def test_three_oracle_forms_agree_on_random_params():
    """Property test (hypothesis): the literal byte-by-byte Writer, the numpy closed form and
    the C restatement agree on random parameters (mask width, seed, min, max) and random
    file lengths, including lengths at min, max and 64 and empty files."""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st

    @settings(max_examples=30, deadline=None, suppress_health_check=list(HealthCheck))
    @given(bits=st.integers(4, 12), seed=st.integers(0, 3), mn=st.integers(64, 3000),
           extra=st.integers(1, 6000), lens=st.lists(st.integers(0, 12_000), min_size=1,
                                                     max_size=12),
           data_seed=st.integers(0, 1 << 30))
    def check(bits, seed, mn, extra, lens, data_seed):
        p = Ch.Params(average_bits=bits, seed=seed, min=mn, max=mn + extra)
        lens = [min(x, 12_000) if x % 7 else [0, mn, mn + extra, 64][x % 4] for x in lens]
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        data = synthetic_bytes(offs, data_seed)
        files = [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(len(lens))]
        lit = Ch.chunk_stream(files, p, "literal")
        fast = Ch.chunk_stream(files, p, "numpy")
        assert [(c.data, c.edge) for c in lit] == [(c.data, c.edge) for c in fast]
        fl = Ch.file_segments_from_chunks(lit, len(files))
        segs, begin = coracle.segment_files(data, offs, p, nthreads=2)
        for f in range(len(files)):
            got = [(int(s["offset"]), int(s["size"]), bytes(s["hash"]))
                   for s in segs[int(begin[f]):int(begin[f + 1])]]
            assert got == fl[f]

    check()
