"""Go 1.16 ``math/rand`` restated in Python — TEST INFRASTRUCTURE (oracle) ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module.  The product (``pfs_amd``) regenerates the same table natively in C++.

Why it is here: the chunker's rolling-hash table is
``buzhash64.GenerateHashes(seed)`` (third-party ``github.com/chmduquesne/rollinghash
v4.0.0+incompatible``, go.mod:13, called at ``src/internal/storage/chunk/option.go:54``),
which draws from Go's stdlib ``math/rand`` (Go 1.16.4, ``etc/compile/GO_VERSION``).
Neither the library nor a Go toolchain exists in this image, so the generator is restated
from its published algorithm:

* ``rngSource`` is an additive lagged-Fibonacci generator over Z/2^64 with
  ``rngLen = 607`` and ``rngTap = 273``; each ``Uint64`` step decrements ``tap`` and
  ``feed`` and stores ``vec[feed] += vec[tap]``.  Re-indexed in time this is
  ``y_t = y_{t-607} + y_{t-273}``, characteristic polynomial ``x^607 - x^334 - 1``.
* ``Seed(s)`` fills ``vec[i] = (x<<40 ^ x'<<20 ^ x'') ^ rngCooked[i]`` from the
  Park-Miller LCG ``x <- 48271 x mod (2^31-1)`` (20 warm-up draws, seed 0 -> 89482311).
* ``rngCooked`` is the state of the same ALFG after 7.8e12 steps from ``srand(1)`` (the
  ``gen_cooked.go`` program, whose seeding uses shifts 20/10).  We regenerate it with a
  polynomial jump-ahead (``x^N mod P`` over Z/2^64) instead of copying Go's table.

Pinned by known answers (tests/test_oracle_kat.py): ``rngCooked[0..1]`` and the Go seed-1
``Int63`` stream 5577006791947779410, 8674665223082153551, 6129484611666145821.
"""
from __future__ import annotations

import functools

RNG_LEN = 607
RNG_TAP = 273
_MASK64 = (1 << 64) - 1
_MASK63 = (1 << 63) - 1
_INT32MAX = (1 << 31) - 1
_COOKED_STEPS = 7_800_000_000_000  # gen_cooked.go: 7.8e12 calls to vrand()


def _seedrand(x: int) -> int:
    # Park-Miller minimal standard, Schrage form in Go; equal to plain modular arithmetic.
    return (48271 * x) % _INT32MAX


def _lcg_fill(seed: int, shifts: tuple[int, int]) -> list[int]:
    """Seed-phase fill shared by gen_cooked.srand (shifts 20/10) and rngSource.Seed (40/20)."""
    seed = seed % _INT32MAX  # Go's % truncates toward zero; fixed below for negatives
    if seed < 0:
        seed += _INT32MAX
    if seed == 0:
        seed = 89482311
    x = seed
    vec = [0] * RNG_LEN
    for i in range(-20, RNG_LEN):
        x = _seedrand(x)
        if i >= 0:
            u = (x << shifts[0]) & _MASK64
            x = _seedrand(x)
            u ^= (x << shifts[1]) & _MASK64
            x = _seedrand(x)
            u ^= x
            vec[i] = u
    return vec


def _go_mod(a: int, m: int) -> int:
    # Go's % on int64 truncates toward zero.
    r = abs(a) % m
    return -r if a < 0 else r


# ---- polynomial jump-ahead over Z/2^64[x] / (x^607 - x^334 - 1) --------------------------

def _polymulmod(a: list[int], b: list[int]) -> list[int]:
    import numpy as np

    # np.convolve on uint64 wraps mod 2^64 (integer multiply-add), which is exactly Z/2^64.
    prod = np.convolve(np.asarray(a, dtype=np.uint64), np.asarray(b, dtype=np.uint64))
    c = [int(v) for v in prod]
    # reduce: x^k = x^(k-607) * (x^334 + 1) for k >= 607, highest first
    for k in range(len(c) - 1, RNG_LEN - 1, -1):
        ck = c[k]
        if ck:
            c[k - RNG_LEN] = (c[k - RNG_LEN] + ck) & _MASK64
            c[k - RNG_TAP] = (c[k - RNG_TAP] + ck) & _MASK64
        c[k] = 0
    return (c + [0] * RNG_LEN)[:RNG_LEN]


def _xpow(n: int) -> list[int]:
    result = [1] + [0] * (RNG_LEN - 1)
    base = [0, 1] + [0] * (RNG_LEN - 2)
    while n:
        if n & 1:
            result = _polymulmod(result, base)
        n >>= 1
        if n:
            base = _polymulmod(base, base)
    return result


def _mulx(c: list[int]) -> list[int]:
    top = c[-1]
    out = [0] + c[:-1]
    if top:
        out[0] = (out[0] + top) & _MASK64
        out[RNG_LEN - RNG_TAP] = (out[RNG_LEN - RNG_TAP] + top) & _MASK64
    return out


def _index_time(i: int) -> int:
    """Sequence index t in [-606, 0] held by vec[i] of a freshly seeded source.

    Step t (t >= 1) writes y_t into vec[(334 - t) mod 607], so the initial vec[i] plays
    the role of y_t for the t <= 0 congruent to 334 - i (vec[334] is y_0, read as the tap
    of step 273 and the feed of step 607)."""
    t = (RNG_LEN - RNG_TAP - i) % RNG_LEN
    return t - RNG_LEN if t > 0 else t


@functools.lru_cache(maxsize=1)
def rng_cooked() -> tuple[int, ...]:
    """Regenerate Go's ``rngCooked[607]`` (as uint64 bit patterns)."""
    vec0 = _lcg_fill(1, (20, 10))
    # initial window y_{-606..0}
    y0 = [0] * RNG_LEN
    for i in range(RNG_LEN):
        y0[_index_time(i) + RNG_LEN - 1] = vec0[i]
    n = _COOKED_STEPS
    # y_{-606+s} = sum_k coef(x^s mod P)_k * y0[k]; we need y_{n-606 .. n}
    c = _xpow(n)  # s = n -> y_{n-606}
    window = []
    for j in range(RNG_LEN):
        window.append(sum(ck * yk for ck, yk in zip(c, y0)) & _MASK64)
        c = _mulx(c)
    # vec[i] after n steps holds y_t for the latest t <= n with feed_t == i
    out = [0] * RNG_LEN
    for i in range(RNG_LEN):
        t = n - ((n - (RNG_LEN - RNG_TAP - i)) % RNG_LEN)
        out[i] = window[t - (n - 606)]
    return tuple(out)


class Source:
    """``rand.NewSource(seed)`` (Go 1.16 rngSource)."""

    def __init__(self, seed: int):
        self.seed(seed)

    def seed(self, seed: int) -> None:
        self.tap = 0
        self.feed = RNG_LEN - RNG_TAP
        s = _go_mod(seed, _INT32MAX)
        if s < 0:
            s += _INT32MAX
        if s == 0:
            s = 89482311
        fill = _lcg_fill(s, (40, 20))
        cooked = rng_cooked()
        self.vec = [fill[i] ^ cooked[i] for i in range(RNG_LEN)]

    def uint64(self) -> int:
        self.tap -= 1
        if self.tap < 0:
            self.tap += RNG_LEN
        self.feed -= 1
        if self.feed < 0:
            self.feed += RNG_LEN
        x = (self.vec[self.feed] + self.vec[self.tap]) & _MASK64
        self.vec[self.feed] = x
        return x

    def int63(self) -> int:
        return self.uint64() & _MASK63


def as_int64(u: int) -> int:
    return u - (1 << 64) if u >> 63 else u
