"""GPU parity of the chunk.Writer mirror (pfs_amd.chunk over the C ABI writer) against the
restated reference Writer (oracle.chunker) on whole annotation streams.

Checks every callback: chunk order, Ref.SizeBytes, Ref.Edge, Ref.Id/Dek (chunk.Create with
CreateOptions{} over the whole chunk, multi-file chunks and chunks spanning writer batches
included), and per annotation the NextDataRef {Hash, OffsetBytes, SizeBytes} — including multi-file chunks (the
buf.Len() >= avg cut before a file, writer.go:118-130), size-0 annotations (E2), the empty
last chunk (E1) and writer batches that split a stream across several GPU scans.
"""
import numpy as np
import pytest

from conftest import fuzz_cases

from oracle import chunker as Ch
from pfs_amd import chunk as pc
from pfs_amd.cdc import synthetic_bytes

pytestmark = pytest.mark.gpu


def run_gpu(files, p: Ch.Params, batch_bytes=1 << 30, writes_per_file=1):
    got = []
    st = pc.Storage(device=0, batch_bytes=batch_bytes)

    def cb(anns):
        got.append([(a.data, None if a.next_data_ref is None else
                     (a.next_data_ref.ref.chunk_index, a.next_data_ref.ref.size_bytes,
                      a.next_data_ref.ref.edge, a.next_data_ref.ref.id,
                      a.next_data_ref.ref.dek, a.next_data_ref.hash,
                      a.next_data_ref.offset_bytes, a.next_data_ref.size_bytes)) for a in anns])

    w = st.new_writer("chunk-writer", cb, pc.with_rolling_hash_config(p.average_bits, p.seed),
                      pc.with_min_max(p.min, p.max))
    for i, f in enumerate(files):
        w.annotate(pc.Annotation(data=i))
        if writes_per_file == 1:
            w.write(f)
        else:
            cuts = sorted(np.random.default_rng(i).integers(0, len(f) + 1, writes_per_file - 1))
            prev = 0
            for c in list(cuts) + [len(f)]:
                w.write(f[prev:c])
                prev = c
    w.close()
    return got, w.chunk_count(), w.annotation_count()


def run_oracle(files, p: Ch.Params):
    chunks = Ch.chunk_stream(files, p, segmenter="numpy", with_ref_id=True)
    out = []
    for ch in chunks:
        out.append([(a.data, None if a.next_data_ref is None else
                     (ch.index, len(ch.data), ch.edge, a.next_data_ref.ref.id,
                      a.next_data_ref.ref.dek, a.next_data_ref.hash,
                      a.next_data_ref.offset_bytes, a.next_data_ref.size_bytes))
                    for a in ch.annotations])
    return out, len(chunks)


def make_files(seed, n, max_len, zero_every=0):
    rng = np.random.default_rng(seed)
    lens = [int(x) for x in rng.integers(0, max_len, n)]
    if zero_every:
        lens = [0 if i % zero_every == 0 else l for i, l in enumerate(lens)]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, seed)
    return [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(n)]


@pytest.mark.parametrize("batch_bytes", [1 << 30, 50_000])
def test_writer_stream_small_params(batch_bytes):
    p = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
    files = make_files(3, 120, 20_000, zero_every=7)
    got, nchunks, nann = run_gpu(files, p, batch_bytes=batch_bytes, writes_per_file=3)
    want, want_n = run_oracle(files, p)
    assert nchunks == want_n and nann == len(files)
    assert got == want


def test_writer_multi_file_chunks_default_params():
    # files below avg accumulate into one chunk until buf.Len() >= 2^23 (writer.go:120)
    p = Ch.Params()
    files = make_files(5, 40, 900_000)
    got, nchunks, _ = run_gpu(files, p)
    want, want_n = run_oracle(files, p)
    assert nchunks == want_n
    assert got == want


def test_writer_stream_ending_on_cut_emits_empty_edge_chunk():
    p = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
    f = make_files(8, 1, 200_000)[0]
    segs = Ch.segments_numpy(f, p)
    cut_end = [s for s in segs if s[2]][-1]
    f = f[:cut_end[0] + cut_end[1]]           # stream now ends exactly on a cut (E1)
    got, nchunks, _ = run_gpu([f], p)
    want, want_n = run_oracle([f], p)
    assert got == want
    assert got[-1] == [(0, None)]             # last chunk is empty, carries no DataRef


def test_writer_refs_chunks_spanning_batches():
    # tiny writer batches: most chunks start in an earlier flush (their bytes are carried)
    p = Ch.Params(average_bits=14, seed=1, min=3000, max=60000)
    files = make_files(12, 60, 9_000, zero_every=5)
    got, nchunks, _ = run_gpu(files, p, batch_bytes=4_000)
    want, want_n = run_oracle(files, p)
    assert nchunks == want_n
    assert got == want
    ids = {d[3] for ch in got for _, d in ch if d is not None}
    assert len(ids) == sum(1 for ch in got if any(d is not None for _, d in ch))


def test_writer_without_ref_ids_leaves_ref_empty():
    p = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
    files = make_files(4, 10, 20_000)
    st = pc.Storage(device=0)
    refs = []
    w = st.new_writer("w", lambda anns: refs.extend(a.next_data_ref.ref for a in anns
                                                     if a.next_data_ref is not None),
                      pc.with_rolling_hash_config(p.average_bits, p.seed),
                      pc.with_min_max(p.min, p.max), pc.without_ref_ids())
    for i, f in enumerate(files):
        w.annotate(pc.Annotation(data=i))
        w.write(f)
    w.close()
    assert refs and all(r.id == b"" and r.dek == b"" for r in refs)


def test_writer_write_before_annotate_is_error():
    from pfs_amd import _lib

    st = pc.Storage(device=0)
    w = st.new_writer("w", None)
    with pytest.raises(_lib.PfsCdcError):
        w.write(b"abc")


@pytest.mark.parametrize("case", fuzz_cases(8))
def test_writer_random_streams_equal_oracle(case):
    """Randomised annotation streams: parameters, file lengths (empty files, files around min,
    avg and max), writer batch sizes and the number of Write calls per file all drawn from a
    seed; every callback must equal the restated Writer's."""
    rng = np.random.default_rng(7000 + case)
    bits = int(rng.integers(8, 15))
    mn = int(rng.integers(64, 6000))
    mx = mn + int(rng.integers(1, 8 * (1 << bits)))
    p = Ch.Params(average_bits=bits, seed=int(rng.integers(0, 4)), min=mn, max=mx)
    kinds = [0, 1, mn - 1, mn, mn + 1, 1 << bits, (1 << bits) + 1, mx - 1, mx, mx + 1]
    lens = []
    for _ in range(int(rng.integers(5, 60))):
        lens.append(int(rng.choice(kinds)) if rng.random() < 0.4 else int(rng.integers(0, 3 * mx)))
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 40 + case)
    files = [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(len(lens))]
    batch = int(rng.choice([2_000, 37_000, 1 << 20, 1 << 30]))
    got, nchunks, nann = run_gpu(files, p, batch_bytes=batch,
                                 writes_per_file=int(rng.integers(1, 5)))
    want, want_n = run_oracle(files, p)
    assert nchunks == want_n and nann == len(files)
    assert got == want
