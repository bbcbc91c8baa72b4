"""GPU parity of the next §8 row: Ref.Id / Ref.Dek of chunk.Create with CreateOptions{}
(/root/reference/src/internal/storage/chunk/transform.go:26-46,173-188; client.go:57):
dek = BLAKE2b-256(BLAKE2b-256(chunk)), id = BLAKE2b-256(ChaCha20_dek(chunk)).

The oracle (oracle/chunker.py create_ref_id, ChaCha20 pinned by RFC 8439 vectors in the CPU
suite) is applied to every segment the GPU produced; the batch form treats each file as its
own writer, so every segment is one chunk."""
import numpy as np
import pytest

from conftest import fuzz_cases

from oracle import chunker as Ch
from oracle import coracle
from pfs_amd.cdc import ChunkParams, Chunker, synthetic_bytes

pytestmark = pytest.mark.gpu

SMALL = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)


def check_refs(res, data, offs, nmax=None):
    assert res.refs is not None and len(res.refs) == len(res.segments)
    idx = range(len(res.segments)) if nmax is None else \
        np.linspace(0, len(res.segments) - 1, nmax).astype(int)
    for i in idx:
        s = res.segments[i]
        a = int(offs[s["file"]]) + int(s["offset"])
        chunk = data[a:a + int(s["size"])].tobytes()
        rid, dek = Ch.create_ref_id(chunk)
        assert bytes(res.refs[i]["dek"]) == dek, f"dek differs at segment {i}"
        assert bytes(res.refs[i]["id"]) == rid, f"id differs at segment {i} (size {len(chunk)})"


def test_ref_ids_small_segments_all_tail_shapes():
    # sizes 1..30000 B: partial ChaCha blocks, partial BLAKE2b blocks, exact multiples
    rng = np.random.default_rng(5)
    lens = np.concatenate([np.arange(1, 200), [63, 64, 65, 127, 128, 129, 191, 192, 193, 255,
                                                256, 257], rng.integers(1, 60_000, 150)])
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 77)
    c = Chunker(ChunkParams(SMALL.average_bits, SMALL.seed, SMALL.min, SMALL.max), 0, ref_ids=True)
    res = c.scan(data, offs)
    segs, _ = coracle.segment_files(data, offs, SMALL, nthreads=8)
    assert np.array_equal(res.segments["hash"], segs["hash"])
    check_refs(res, data, offs)


def test_ref_ids_default_params_multi_mib():
    offs = np.array([0, 3 << 20, (3 << 20) + 12345, (12 << 20) + 7, (40 << 20) + 999],
                    dtype=np.uint64)
    data = synthetic_bytes(offs, 11)
    c = Chunker(ChunkParams(), 0, ref_ids=True)
    res = c.scan(data, offs)
    check_refs(res, data, offs)


def test_ref_ids_device_resident_batch_and_toggle():
    import torch
    offs = (np.arange(65, dtype=np.uint64) * np.uint64(1_500_001))
    c = Chunker(ChunkParams(), 0)
    t = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
    c.fill_synthetic(t, offs, 0xC2)
    plain = c.scan(t, offs)
    assert plain.refs is None
    c.set_ref_ids(True)
    res = c.scan(t, offs)
    assert np.array_equal(res.segments, plain.segments)  # refs do not disturb the records
    check_refs(res, t.cpu().numpy(), offs, nmax=24)
    assert c.timings()["ref_ids"] > 0


def _encrypt(chunks):
    """Stored form of each chunk (chunk.Create, CreateOptions{}): ChaCha20_dek(chunk)."""
    out, refs = [], np.zeros(len(chunks), dtype=[("id", "u1", (32,)), ("dek", "u1", (32,))])
    for i, ch in enumerate(chunks):
        rid, dek = Ch.create_ref_id(ch)
        out.append(Ch.chacha20_xor(dek, ch))
        refs[i]["id"] = np.frombuffer(rid, dtype=np.uint8)
        refs[i]["dek"] = np.frombuffer(dek, dtype=np.uint8)
    return out, refs


def test_get_chunks_decrypts_and_verifies():
    rng = np.random.default_rng(9)
    lens = [0, 1, 63, 64, 65, 127, 128, 129, 1000, 4096, 70_001, 1 << 20] + \
        list(rng.integers(1, 300_000, 40))
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    plain = synthetic_bytes(offs, 31)
    chunks = [plain[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(len(lens))]
    ctexts, refs = _encrypt(chunks)
    stored = np.frombuffer(b"".join(ctexts), dtype=np.uint8).copy()
    c = Chunker(ChunkParams(), 0)
    pt, ok = c.get_chunks(stored, offs, refs)
    assert ok.all()
    assert np.array_equal(pt, plain)
    # a flipped stored byte fails verification of exactly that chunk (verifyData)
    bad = stored.copy()
    k = 7
    bad[int(offs[k]) + 3] ^= 0x40
    pt2, ok2 = c.get_chunks(bad, offs, refs)
    assert not ok2[k] and ok2.sum() == len(lens) - 1


def test_get_chunks_device_resident_roundtrip_of_scan_refs():
    # write path (scan + Ref.Id) then read path (get_chunks) on the same segments
    import torch
    offs = (np.arange(9, dtype=np.uint64) * np.uint64(3_000_017))
    c = Chunker(ChunkParams(), 0, ref_ids=True)
    t = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
    c.fill_synthetic(t, offs, 0xC4)
    res = c.scan(t, offs)
    host = t.cpu().numpy()
    chunks = [host[int(offs[s["file"]]) + int(s["offset"]):][:int(s["size"])].tobytes()
              for s in res.segments]
    ctexts = [Ch.chacha20_xor(bytes(r["dek"]), ch) for r, ch in zip(res.refs, chunks)]
    coffs = np.concatenate([[0], np.cumsum([len(x) for x in chunks])]).astype(np.uint64)
    dev_ct = torch.from_numpy(np.frombuffer(b"".join(ctexts), dtype=np.uint8).copy()).cuda()
    out = torch.empty_like(dev_ct)
    _, ok = c.get_chunks(dev_ct, coffs, res.refs, out=out)
    assert ok.all()
    assert np.array_equal(out.cpu().numpy(), np.frombuffer(b"".join(chunks), dtype=np.uint8))


# ---------------------------------------------------------------- chunk formation + Create

@pytest.mark.parametrize("split", [0, 1])
def test_create_refs_matches_oracle_with_known_hashes(split, knob):
    # split 1: ChaCha20 pass (coalesced: keystream parked in LDS, 16-byte pieces per lane)
    # + BLAKE2b of the ciphertext; 0: the fused pass
    knob("PFSCDC_REFID_SPLIT", split)
    rng = np.random.default_rng(21)
    lens = [0, 1, 63, 64, 65, 127, 128, 129, 5000, (3 << 20) + 5] + \
        list(rng.integers(1, 400_000, 60))
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 41)
    chunks = [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(len(lens))]
    c = Chunker(ChunkParams(), 0)
    refs, hashes = c.create_refs(data, offs)
    for i, ch in enumerate(chunks):
        assert bytes(hashes[i]) == Ch.blake2b256(ch)
        assert (bytes(refs[i]["id"]), bytes(refs[i]["dek"])) == Ch.create_ref_id(ch), i
    # every other content hash supplied by the caller: same refs, supplied hashes kept
    known = (np.arange(len(lens)) % 2).astype(np.uint8)
    given = np.where(known[:, None] == 1, hashes, 0).astype(np.uint8)
    refs2, hashes2 = c.create_refs(data, offs, given, known)
    assert np.array_equal(refs2, refs) and np.array_equal(hashes2, hashes)


def _oracle_streams(files, p, streams):
    """Chunks of each stream (one chunk.Writer per stream) with Ref ids, in order."""
    out = []
    for b, e in zip(streams[:-1], streams[1:]):
        if e > b:
            out.extend(Ch.chunk_stream(files[b:e], p, with_ref_id=True))
    return out


@pytest.mark.parametrize("streams", [None, [0, 17, 17, 60, 95, 120]])
def test_form_chunks_and_refs_match_writer_streams(streams):
    import torch
    p = Ch.Params(average_bits=13, seed=1, min=3000, max=40000)
    rng = np.random.default_rng(3)
    lens = [0 if i % 9 == 0 else int(x) for i, x in enumerate(rng.integers(0, 25_000, 120))]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    c = Chunker(ChunkParams(p.average_bits, p.seed, p.min, p.max), 0)
    t = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
    c.fill_synthetic(t, offs, 0x5F)
    host = t.cpu().numpy()
    files = [host[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(len(lens))]
    c.scan(t, offs)
    coffs, hashes, known = c.form_chunks(streams)
    want = _oracle_streams(files, p, streams or [0, len(lens)])
    assert len(coffs) - 1 == len(want)
    assert [int(b - a) for a, b in zip(coffs[:-1], coffs[1:])] == [len(ch.data) for ch in want]
    assert coffs[0] == 0 and coffs[-1] == offs[-1]
    for i, ch in enumerate(want):
        assert bytes(host[int(coffs[i]):int(coffs[i + 1])]) == ch.data
        pieces = [a for a in ch.annotations if a.next_data_ref is not None]
        assert known[i] == (len(pieces) == 1 and len(ch.data) > 0)
        if known[i]:
            assert bytes(hashes[i]) == Ch.blake2b256(ch.data)
    refs, _ = c.create_refs(t, coffs, hashes, known)
    for i, ch in enumerate(want):
        rid, dek = Ch.create_ref_id(ch.data)
        assert bytes(refs[i]["id"]) == rid and bytes(refs[i]["dek"]) == dek, i


@pytest.mark.parametrize("case", fuzz_cases(4))
def test_get_chunks_random_tampering(case):
    """chunk.Get (verify BLAKE2b(stored) == Ref.Id, then decrypt) on random chunk sizes with
    a random subset damaged: a flipped stored byte anywhere (first, last, inside a partial
    final block) or a Ref.Id that names other bytes.  Exactly the damaged chunks fail, and
    every other chunk decrypts to its plaintext."""
    rng = np.random.default_rng(9900 + case)
    lens = [int(rng.choice([0, 1, 127, 128, 129, 255, 256, 257])) if rng.random() < 0.3 else
            int(rng.integers(1, 200_000)) for _ in range(int(rng.integers(10, 60)))]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    plain = synthetic_bytes(offs, 50 + case)
    chunks = [plain[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(len(lens))]
    ctexts, refs = _encrypt(chunks)
    stored = np.frombuffer(b"".join(ctexts), dtype=np.uint8).copy()
    orig, refs = refs, refs.copy()
    bad = set()
    for i in range(len(lens)):
        if lens[i] == 0 or rng.random() > 0.3:
            continue
        bad.add(i)
        if rng.random() < 0.7:
            pos = int(rng.choice([0, lens[i] - 1, int(rng.integers(0, lens[i]))]))
            stored[int(offs[i]) + pos] ^= 1 << int(rng.integers(0, 8))
        else:
            refs[i]["id"] = refs[(i + 1) % len(lens)]["id"] if lens[(i + 1) % len(lens)] \
                else np.frombuffer(bytes(32), dtype=np.uint8)
            if bytes(refs[i]["id"]) == bytes(orig[i]["id"]):
                bad.discard(i)  # an identical neighbour: the id still names these bytes
    c = Chunker(ChunkParams(), 0)
    pt, ok = c.get_chunks(stored, offs, refs)
    assert set(np.flatnonzero(~ok.astype(bool)).tolist()) == bad
    for i in range(len(lens)):
        if i not in bad:
            assert np.array_equal(pt[int(offs[i]):int(offs[i + 1])],
                                  plain[int(offs[i]):int(offs[i + 1])]), i
    c.close()
