"""buzhash64 (rollinghash v4.0.0) restated in Python — TEST INFRASTRUCTURE (oracle) ONLY.

Third-party dependency of the reference: ``github.com/chmduquesne/rollinghash
v4.0.0+incompatible`` (``go.mod:13``, ``go.sum:183``), not vendored under /root/reference.
Call sites restated here: ``chunk/option.go:54`` (``NewFromUint64Array(GenerateHashes(seed))``),
``chunk/writer.go:100-103`` (``Reset`` + ``Write(initialWindow)``), ``writer.go:166-167``
(``Roll`` + ``Sum64``) and ``chunk_test.go:125-137``.

Assumptions, stated so a reviewer with Go can check them:

* A1 ``GenerateHashes(seed)``: ``r := rand.New(rand.NewSource(seed))``; for i in 0..255 draw
  ``x := uint64(r.Int63())`` until ``x`` was not drawn before; ``T[i] = x``.
* A2 ``Write(w)`` sets the window to ``w`` and folds ``sum = rotl(sum,1) ^ T[c]`` for every c;
  ``Roll(c)`` does ``sum = rotl(sum,1) ^ rotl(T[out], len(w) % 64) ^ T[c]`` and replaces the
  oldest window byte.  Go's ``x >> 64 == 0`` makes the len%64 == 0 rotation the identity (E4).
"""
from __future__ import annotations

from . import gorand

_M64 = (1 << 64) - 1


def generate_hashes(seed: int, draw: str = "int63") -> list[int]:
    """A1: ``draw="int63"`` (T[i] = uint64(rand.Int63()), what the product implements).
    ``draw="uint64"`` is the one plausible alternative (T[i] = rand.Uint64(), the full 64-bit
    ALFG value); oracle/go_probe prints the real GenerateHashes so a Go run picks one."""
    if draw not in ("int63", "uint64"):
        raise ValueError(draw)
    r = gorand.Source(seed)
    nxt = r.int63 if draw == "int63" else r.uint64
    used: set[int] = set()
    out = []
    for _ in range(256):
        x = nxt()
        while x in used:
            x = nxt()
        used.add(x)
        out.append(x)
    return out


def rotl(x: int, k: int) -> int:
    k %= 64
    if k == 0:
        return x
    return ((x << k) | (x >> (64 - k))) & _M64


class Buzhash64:
    def __init__(self, table: list[int]):
        self.t = list(table)
        self.reset()

    def reset(self) -> None:
        self.sum = 0
        self.window = bytearray()
        self.oldest = 0

    def write(self, data: bytes) -> None:
        n = len(data) or 1
        self.window = bytearray(data) if data else bytearray(1)
        assert len(self.window) == n
        for c in self.window:
            self.sum = rotl(self.sum, 1) ^ self.t[c]
        self.oldest = 0
        self.n_rotate = len(self.window) % 64

    def roll(self, c: int) -> None:
        hn = self.t[c]
        ho = self.t[self.window[self.oldest]]
        self.window[self.oldest] = c
        self.oldest += 1
        if self.oldest >= len(self.window):
            self.oldest = 0
        self.sum = rotl(self.sum, 1) ^ rotl(ho, self.n_rotate) ^ hn

    def sum64(self) -> int:
        return self.sum
