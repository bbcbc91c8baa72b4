"""Known-answer tests that pin the oracle's components (CPU only).

* Go 1.16 math/rand: rngCooked[0..1] (Go's math/rand/rng.go table) and the famous seed-1
  Int63 stream (Go playground ``rand.Int()``), SURVEY.md §8c.
* buzhash64.GenerateHashes(1): T[0], T[1], T[255] (SURVEY.md §8c probe values).
* BLAKE2b: RFC 7693 Appendix A ("abc", BLAKE2b-512) and the empty-string BLAKE2b-256 digest
  (FileInfo.Hash of a zero-byte file, E2).
* ChaCha20: RFC 8439 §2.3.2 (block function) and §2.4.2 (encryption) test vectors.
"""
import hashlib

import numpy as np

from oracle import buzhash64, chunker, coracle, gorand

GO_SEED1_INT63 = [5577006791947779410, 8674665223082153551, 6129484611666145821,
                  4037200794235010051, 3916589616287113937]


def test_rng_cooked_head():
    c = gorand.rng_cooked()
    assert gorand.as_int64(c[0]) == -4181792142133755926
    assert gorand.as_int64(c[1]) == -4576982950128230565


def test_go_seed1_int63_stream():
    s = gorand.Source(1)
    assert [s.int63() for _ in range(5)] == GO_SEED1_INT63


def test_generate_hashes_seed1():
    t = buzhash64.generate_hashes(1)
    assert t[0] == 5577006791947779410
    assert t[1] == 8674665223082153551
    assert t[255] == 3062676815688632933
    assert len(set(t)) == 256 and all(x < (1 << 63) for x in t)


def test_seed0_is_go_default_89482311():
    # rand.NewSource(0) seeds like 89482311 (rng.go Seed: seed == 0 -> 89482311)
    a, b = gorand.Source(0), gorand.Source(89482311)
    assert [a.int63() for _ in range(4)] == [b.int63() for _ in range(4)]


def test_blake2b_rfc7693_and_empty():
    want512 = ("ba80a53f981c4d0d6a2797b69f12f6e94c212f14685ac4b74b12bb6fdbffa2d1"
               "7d87c5392aab792dc252d5de4533cc9518d38aa8dbf1925ab92386edd4009923")
    assert hashlib.blake2b(b"abc").hexdigest() == want512
    empty = "0e5751c026e543b2e8ab2eb06099daa1d1e5df47778f7787faab45cdf12fe3a8"
    assert chunker.blake2b256(b"").hex() == empty
    assert coracle.blake2b256(b"").hex() == empty


def test_c_oracle_blake2b_matches_hashlib_block_edges():
    rng = np.random.default_rng(0)
    for n in [1, 64, 127, 128, 129, 255, 256, 257, 1000, 65536 + 3]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert coracle.blake2b256(d) == hashlib.blake2b(d, digest_size=32).digest()


def test_chacha20_rfc8439():
    # §2.3.2 block function: key 00..1f, nonce 000000090000004a00000000, counter 1
    key = bytes(range(32))
    # our keystream fixes nonce = 0 (transform.go uses a zero nonce); check §2.4.2-style
    # with zero nonce via the A.1 vector #1: all-zero key, counter 0 -> known keystream
    ks = chunker._chacha20_keystream(bytes(32), 64)
    assert ks.hex() == ("76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
                        "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586")
    # A.1 vector #2: all-zero key, counter 1
    ks1 = chunker._chacha20_keystream(bytes(32), 64, counter0=1)
    assert ks1.hex() == ("9f07e7be5551387a98ba977c732d080dcb0f29a048e3656912c6533e32ee7aed"
                         "29b721769ce64e43d57133b074d839d531ed1f28510afb45ace10a1f4b794d6f")
    assert len(key) == 32
