"""GPU parity of pfscdc_commit_refs, the commit data plane's hashing in one pass: a
cuts-only scan (PFSCDC_OPT_CUTS_ONLY), pfscdc_form_chunks, then one BLAKE2b launch over every
segment (DataRef.Hash, writer.go:301-312) and every multi-DataRef chunk (chunk content hash,
writer.go:233-253) followed by chunk.Create (transform.go:26-46,173-188).  Bar: bit-identical
to the separate passes (scan with segment hashes, pfscdc_create_refs), which the other GPU
suites check against the oracle, and to the oracle directly on a sample."""
import hashlib

import numpy as np
import pytest

from conftest import fuzz_cases

from oracle import chunker as Ch
from pfs_amd.cdc import ChunkParams, Chunker, synthetic_bytes

pytestmark = pytest.mark.gpu


def both_ways(p: Ch.Params, offs, streams, data):
    cp = ChunkParams(p.average_bits, p.seed, p.min, p.max)
    a = Chunker(cp, 0)
    ra = a.scan(data, offs)
    coffs, hashes, known = a.form_chunks(streams)
    refs_a, chash_a = a.create_refs(data, coffs, hashes, known)
    b = Chunker(cp, 0)
    b.set_cuts_only(True)
    rb = b.scan(data, offs)
    for f in ("offset", "size", "file", "flags"):
        assert np.array_equal(rb.segments[f], ra.segments[f]), f"segment {f} differs" 
    coffs_b, _, known_b = b.form_chunks(streams)
    assert np.array_equal(coffs_b, coffs) and np.array_equal(known_b, known)
    refs_b, chash_b, seg_b = b.commit_refs(data, coffs_b, known_b)
    assert np.array_equal(seg_b, ra.segments["hash"]), "DataRef hashes differ"
    assert np.array_equal(chash_b, chash_a), "chunk content hashes differ"
    assert np.array_equal(refs_b["id"], refs_a["id"]) and np.array_equal(refs_b["dek"], refs_a["dek"])
    a.close()
    b.close()
    return coffs, known, refs_b, chash_b, ra


@pytest.mark.parametrize("seed", [1, 2])
def test_commit_refs_equal_separate_passes_small_params(seed):
    # many multi-DataRef chunks: small files under a 4 KiB .. 60 KB chunker, three streams
    p = Ch.Params(average_bits=13, seed=1, min=4000, max=60000)
    rng = np.random.default_rng(seed)
    lens = np.concatenate([rng.integers(0, 9000, 300), [0, 1, 3999, 4000, 60000, 60001],
                           rng.integers(20_000, 200_000, 40)])
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 300 + seed)
    nf = len(lens)
    streams = [0, nf // 3, nf // 3, 2 * nf // 3, nf]  # an empty stream too
    coffs, known, refs, chash, _ = both_ways(p, offs, streams, data)
    assert (~known.astype(bool)).sum() > 20
    for i in np.linspace(0, len(coffs) - 2, 12).astype(int):
        chunk = data[int(coffs[i]):int(coffs[i + 1])].tobytes()
        assert bytes(chash[i]) == hashlib.blake2b(chunk, digest_size=32).digest()
        rid, dek = Ch.create_ref_id(chunk)
        assert bytes(refs[i]["id"]) == rid and bytes(refs[i]["dek"]) == dek


def test_commit_refs_default_params_device_resident():
    import torch

    p = Ch.Params()
    lens = [3 << 20, 12345, (9 << 20) + 7, 999_999, 1_000_000, 0, (21 << 20) + 5, 4 << 20]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    c = Chunker(ChunkParams(), 0)
    t = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
    c.fill_synthetic(t, offs, 0xC4)
    both_ways(p, offs, [0, 3, len(lens)], t)
    c.close()


def test_commit_refs_needs_a_cuts_only_scan():
    from pfs_amd import _lib

    p = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
    offs = np.array([0, 50_000, 90_000], dtype=np.uint64)
    data = synthetic_bytes(offs, 5)
    c = Chunker(ChunkParams(p.average_bits, p.seed, p.min, p.max), 0)
    c.scan(data, offs)
    coffs, _, known = c.form_chunks()
    with pytest.raises(_lib.PfsCdcError):
        c.commit_refs(data, coffs, known)
    c.close()


def test_commit_refs_rejects_a_known_chunk_that_is_no_segment():
    """hash_known marks a chunk whose content hash is its one segment's; a chunk of several
    DataRefs marked known matches no scan segment exactly and must be refused (EINVAL), not
    given a neighbouring segment's hash."""
    from pfs_amd import _lib

    p = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
    lens = [700, 900, 1500, 20_000, 300, 300, 45_000, 800]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 17)
    c = Chunker(ChunkParams(p.average_bits, p.seed, p.min, p.max), 0)
    c.set_cuts_only(True)
    c.scan(data, offs)
    coffs, _, known = c.form_chunks()
    multi = np.flatnonzero(known == 0)
    assert len(multi), "the layout must form a multi-DataRef chunk"
    bad = known.copy()
    bad[multi[0]] = 1
    with pytest.raises(_lib.PfsCdcError, match="not one segment"):
        c.commit_refs(data, coffs, bad)
    c.close()


def test_commit_refs_ciphertext_in_place():
    """PFSCDC_OPT_CTEXT_IN_PLACE: the same Refs as the copy form, and the device buffer then
    holds every chunk's ChaCha20_dek(chunk) (transform.go:181-188), the object chunk.Create
    uploads: BLAKE2b of it is Ref.Id (client.go:57), and the oracle's cipher gives the same
    bytes on a sample."""
    import torch

    p = Ch.Params(average_bits=13, seed=1, min=4000, max=60000)
    rng = np.random.default_rng(7)
    lens = np.concatenate([rng.integers(0, 9000, 200), rng.integers(20_000, 150_000, 30)])
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    host = synthetic_bytes(offs, 77)
    nf = len(lens)
    streams = [0, nf // 2, nf]
    cp = ChunkParams(p.average_bits, p.seed, p.min, p.max)
    a = Chunker(cp, 0)
    a.set_cuts_only(True)
    ta = torch.from_numpy(host).to("cuda:0")
    a.scan(ta, offs)
    coffs, _, known = a.form_chunks(streams)
    refs_a, chash_a, seg_a = a.commit_refs(ta, coffs, known)
    assert torch.equal(ta.cpu(), torch.from_numpy(host)), "the copy form left the input alone"
    b = Chunker(cp, 0)
    b.set_cuts_only(True)
    b.set_ctext_in_place(True)
    tb = torch.from_numpy(host).to("cuda:0")
    b.scan(tb, offs)
    coffs_b, _, known_b = b.form_chunks(streams)
    refs_b, chash_b, seg_b = b.commit_refs(tb, coffs_b, known_b)
    assert np.array_equal(refs_b["id"], refs_a["id"]) and np.array_equal(refs_b["dek"], refs_a["dek"])
    assert np.array_equal(chash_b, chash_a) and np.array_equal(seg_b, seg_a)
    ct = tb.cpu().numpy()
    for i in range(len(coffs) - 1):
        c = ct[int(coffs[i]):int(coffs[i + 1])].tobytes()
        assert hashlib.blake2b(c, digest_size=32).digest() == bytes(refs_b[i]["id"]), i
    for i in np.linspace(0, len(coffs) - 2, 6).astype(int):
        plain = host[int(coffs[i]):int(coffs[i + 1])].tobytes()
        assert ct[int(coffs[i]):int(coffs[i + 1])].tobytes() == Ch.chacha20_xor(
            bytes(refs_b[i]["dek"]), plain), i
    a.close()
    b.close()


def test_ciphertext_in_place_needs_device_bytes():
    from pfs_amd import _lib

    p = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
    offs = np.array([0, 50_000, 90_000], dtype=np.uint64)
    data = synthetic_bytes(offs, 5)
    c = Chunker(ChunkParams(p.average_bits, p.seed, p.min, p.max), 0)
    c.set_cuts_only(True)
    c.set_ctext_in_place(True)
    c.scan(data, offs)
    coffs, _, known = c.form_chunks()
    with pytest.raises(_lib.PfsCdcError, match="device bytes"):
        c.commit_refs(data, coffs, known)
    c.close()


@pytest.mark.parametrize("in_place", [False, True])
def test_commit_refs_two_chunk_sets_equal_one_pass(in_place, knob):
    """The two-set commit (the long chunks' hashes and chunk.Create on the ctx stream at issue
    priority, the rest on a helper context beside them, PFSCDC_COMMIT_TWO_SETS) gives the same
    DataRef hashes, content hashes, Refs and ciphertext as the one-pass form, at several
    split points (PFSCDC_COMMIT_LONG_PCT), and the oracle's Ref.Id on a sample."""
    import torch

    p = Ch.Params(average_bits=13, seed=1, min=4000, max=60000)
    rng = np.random.default_rng(11)
    lens = np.concatenate([rng.integers(0, 9000, 250), [0, 0, 60000, 60001, 1],
                           rng.integers(20_000, 250_000, 40)])
    rng.shuffle(lens)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    host = synthetic_bytes(offs, 91)
    nf = len(lens)
    streams = [0, nf // 4, nf // 2, nf]
    cp = ChunkParams(p.average_bits, p.seed, p.min, p.max)

    def run(two_sets, pct):
        knob("PFSCDC_COMMIT_TWO_SETS", 1 if two_sets else 0)
        knob("PFSCDC_COMMIT_LONG_PCT", pct)
        c = Chunker(cp, 0)
        c.set_cuts_only(True)
        c.set_ctext_in_place(in_place)
        t = torch.from_numpy(host).to("cuda:0")
        c.scan(t, offs)
        coffs, _, known = c.form_chunks(streams)
        refs, chash, seg = c.commit_refs(t, coffs, known)
        c.close()
        return coffs, known, refs, chash, seg, t.cpu().numpy()

    base = run(False, 50)
    coffs, known, refs0, chash0, seg0, buf0 = base
    sizes = np.diff(coffs)
    assert (~known.astype(bool)).sum() > 10 and (sizes > 0.5 * sizes.max()).sum() > 1
    for pct in (10, 50, 90):
        _, _, refs, chash, seg, buf = run(True, pct)
        assert np.array_equal(seg, seg0), pct
        assert np.array_equal(chash, chash0), pct
        assert np.array_equal(refs["id"], refs0["id"]) and np.array_equal(refs["dek"], refs0["dek"]), pct
        assert np.array_equal(buf, buf0), pct  # the plaintext left alone, or the same ciphertext
    for i in np.linspace(0, len(coffs) - 2, 8).astype(int):
        chunk = host[int(coffs[i]):int(coffs[i + 1])].tobytes()
        rid, dek = Ch.create_ref_id(chunk)
        assert bytes(refs0[i]["id"]) == rid and bytes(refs0[i]["dek"]) == dek


@pytest.mark.parametrize("refid_split", [0, 1])
def test_ciphertext_in_place_whatever_the_refid_form(refid_split, knob):
    """In place, chunk.Create always takes the split Ref.Id form: the fused kernel's plaintext
    and ciphertext pointers are __restrict__ and must not alias, so the PFSCDC_REFID_SPLIT knob at 0 (or a
    chunk count above the quads, which picks the fused form) must not reach it with
    ctext_out == data.  Refs and the buffer equal the copy form's."""
    import torch

    p = Ch.Params(average_bits=13, seed=1, min=4000, max=60000)
    rng = np.random.default_rng(23)
    lens = np.concatenate([rng.integers(0, 9000, 150), rng.integers(20_000, 150_000, 25)])
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    host = synthetic_bytes(offs, 23)
    streams = [0, len(lens) // 2, len(lens)]
    cp = ChunkParams(p.average_bits, p.seed, p.min, p.max)
    knob("PFSCDC_COMMIT_TWO_SETS", 0)

    def run(in_place, split):
        knob("PFSCDC_REFID_SPLIT", split)
        c = Chunker(cp, 0)
        c.set_cuts_only(True)
        c.set_ctext_in_place(in_place)
        t = torch.from_numpy(host).to("cuda:0")
        c.scan(t, offs)
        coffs, _, known = c.form_chunks(streams)
        refs, chash, seg = c.commit_refs(t, coffs, known)
        c.close()
        return coffs, refs, chash, seg, t.cpu().numpy()

    coffs, refs0, chash0, seg0, _ = run(False, -1)
    _, refs, chash, seg, ct = run(True, refid_split)
    assert np.array_equal(refs["id"], refs0["id"]) and np.array_equal(refs["dek"], refs0["dek"])
    assert np.array_equal(chash, chash0) and np.array_equal(seg, seg0)
    for i in range(len(coffs) - 1):
        c = ct[int(coffs[i]):int(coffs[i + 1])].tobytes()
        assert hashlib.blake2b(c, digest_size=32).digest() == bytes(refs[i]["id"]), i


@pytest.mark.parametrize("case", fuzz_cases(6))
def test_commit_random_layouts_equal_oracle(knob, case):
    """Randomised commits: parameters, file lengths (empty, around min and max, multi-MB),
    stream borders (empty streams included) and the commit's forms (one or two chunk sets,
    fused or split Ref.Id pass) drawn per case.  Chunk boundaries equal the restated Writer's
    per stream, every chunk's content hash equals hashlib's, and a sample of Ref.Ids the
    oracle's chunk.Create."""
    rng = np.random.default_rng(4400 + case)
    bits = int(rng.integers(12, 17))
    mn = int(rng.integers(1000, 20_000))
    p = Ch.Params(average_bits=bits, seed=int(rng.integers(0, 3)), min=mn,
                  max=mn + int(rng.integers(1, 6 * (1 << bits))))
    knob("PFSCDC_COMMIT_TWO_SETS", int(rng.integers(-1, 2)))
    knob("PFSCDC_REFID_SPLIT", int(rng.integers(-1, 2)))
    kinds = [0, 1, p.min - 1, p.min, p.max, p.max + 1, 1 << bits]
    lens = [int(rng.choice(kinds)) if rng.random() < 0.3 else
            int(rng.integers(0, 2 * p.max if rng.random() < 0.8 else 30 * p.max))
            for _ in range(int(rng.integers(20, 200)))]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 700 + case)
    nf = len(lens)
    inner = sorted(int(x) for x in rng.integers(0, nf + 1, int(rng.integers(0, 5))))
    streams = [0] + inner + [nf]
    coffs, known, refs, chash, _ = both_ways(p, offs, streams, data)
    want = []
    for a, b in zip(streams[:-1], streams[1:]):
        files = [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(a, b)]
        want += [len(ch.data) for ch in Ch.chunk_stream(files, p)] if files else []
    assert np.diff(coffs).tolist() == want
    for i in range(len(coffs) - 1):
        chunk = data[int(coffs[i]):int(coffs[i + 1])].tobytes()
        assert bytes(chash[i]) == hashlib.blake2b(chunk, digest_size=32).digest(), i
    for i in np.linspace(0, len(coffs) - 2, 8).astype(int):
        rid, dek = Ch.create_ref_id(data[int(coffs[i]):int(coffs[i + 1])].tobytes())
        assert bytes(refs[i]["id"]) == rid and bytes(refs[i]["dek"]) == dek, i
    if rng.random() < 0.5:  # the ciphertext written over device-resident input
        import torch

        cp = ChunkParams(p.average_bits, p.seed, p.min, p.max)
        c = Chunker(cp, 0)
        c.set_cuts_only(True)
        c.set_ctext_in_place(True)
        t = torch.from_numpy(data).to("cuda:0")
        c.scan(t, offs)
        coffs_c, _, known_c = c.form_chunks(streams)
        refs_c, _, _ = c.commit_refs(t, coffs_c, known_c)
        assert np.array_equal(refs_c["id"], refs["id"]) and np.array_equal(refs_c["dek"], refs["dek"])
        ct = t.cpu().numpy()
        for i in range(len(coffs) - 1):
            blob = ct[int(coffs[i]):int(coffs[i + 1])].tobytes()
            assert hashlib.blake2b(blob, digest_size=32).digest() == bytes(refs[i]["id"]), i
        c.close()
