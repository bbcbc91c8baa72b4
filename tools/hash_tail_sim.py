"""Event simulation of the hash kernel's drain on configs[1] (c2) steps: which queue policy
ends the launch soonest.  Model: 1024 SIMDs x 2 waves x 16 quads; a wave
advances one 128-B block per C2 cycles while its SIMD-mate is active at the same priority,
per C1 cycles alone or when it outranks the mate (s_setprio 2 while a quad has more than
T blocks left), and gets what is left of the SIMD otherwise.  Chains are drawn from the
launch-wide queue in its order when a quad frees.  Segment sizes follow the cut rule on
4 MiB files (min 1,000,000, candidates at rate 2^-23 per position)."""
import heapq
import sys

import numpy as np

C2 = 2 * 2205.0   # cycles per block per wave, two waves sharing a SIMD (4.06 cycles/instr)
C1 = 2556.0       # a lone wave (lone-chain measurement)
GHZ = 2.2


def c2_segments(nfiles=32768, fb=4 << 20, mn=1_000_000, bits=23, seed=1):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(nfiles):
        pos = 0
        while fb - pos > 0:
            c = pos + mn - 1 + int(rng.exponential(2 ** bits))  # first candidate past min
            if c + 1 >= fb:
                out.append(fb - pos)
                break
            out.append(c + 1 - pos)
            pos = c + 1
    return np.array(out, dtype=np.int64)


def simulate(sizes, order="lpt", prio_T=8192, nsimd=1024, wps=2, qpw=16, tail_from_back=None):
    blocks = (sizes + 127) // 128
    if order == "lpt":
        q = list(np.sort(blocks)[::-1])
    else:
        q = list(blocks)
    head, tail = 0, len(q)  # queue [head, tail)
    W = nsimd * wps
    prog = np.zeros(W)            # blocks advanced (all quads of a wave advance together)
    ends = [[] for _ in range(W)]  # per wave: chain end progress of its active quads
    rate = np.zeros(W)
    t_last = np.zeros(W)           # time prog was last brought up to date
    alive = np.ones(W, bool)
    ver = np.zeros(W, np.int64)
    total_work = blocks.sum()

    def take(w):
        nonlocal head, tail
        if head >= tail:
            return None
        if tail_from_back is not None and tail_from_back(w, prog[w], head, tail, q):
            tail -= 1
            return q[tail]
        head += 1
        return q[head - 1]

    for w in range(W):  # initial fill
        for _ in range(qpw):
            b = take(w)
            if b is None:
                break
            ends[w].append(b)
    def hi(w):
        return prio_T > 0 and any(e - prog[w] > prio_T for e in ends[w])

    def simd_rates(s, t):
        ws = [w for w in range(s * wps, s * wps + wps) if alive[w] and ends[w]]
        for w in range(s * wps, s * wps + wps):
            prog[w] += rate[w] * (t - t_last[w])
            t_last[w] = t
            rate[w] = 0.0
        if len(ws) == 1:
            rate[ws[0]] = 1.0 / C1
        elif len(ws) == 2:
            a, b = ws
            pa, pb = hi(a), hi(b)
            if pa == pb:
                rate[a] = rate[b] = 1.0 / C2
            else:
                top, low = (a, b) if pa else (b, a)
                rate[top] = 1.0 / C1
                rate[low] = max(2.0 / C2 - 1.0 / C1, 0.0)
        return ws

    ev = []

    def schedule(w, t):
        ver[w] += 1
        if not ends[w] or rate[w] <= 0:
            return
        nxt = min(ends[w])
        if prio_T > 0:
            for e in ends[w]:
                if e - prog[w] > prio_T:  # the crossing, strictly past it
                    nxt = min(nxt, e - prio_T + 0.5)
        heapq.heappush(ev, (t + max(nxt - prog[w], 0.0) / rate[w], ver[w], w))

    for s in range(nsimd):
        for w in simd_rates(s, 0.0):
            schedule(w, 0.0)
    simd_end = np.zeros(nsimd)
    wave_end = np.zeros(W)
    while ev:
        t, v, w = heapq.heappop(ev)
        if v != ver[w]:
            continue
        s = w // wps
        prog[w] += rate[w] * (t - t_last[w])
        t_last[w] = t
        eps = 1e-6
        done = [e for e in ends[w] if e <= prog[w] + eps]
        ends[w] = [e for e in ends[w] if e > prog[w] + eps]
        for _ in done:
            b = take(w)
            if b is not None:
                ends[w].append(prog[w] + b)
        if not ends[w]:
            alive[w] = False
            wave_end[w] = t
        for x in simd_rates(s, t):
            schedule(x, t)
        if not any(alive[s * wps:(s + 1) * wps] & np.array([bool(ends[x]) for x in range(s * wps, (s + 1) * wps)])):
            simd_end[s] = max(simd_end[s], t)
    span = simd_end.max()
    idle = 1.0 - simd_end.sum() / (span * nsimd)
    ms = lambda c: c / GHZ / 1e6
    ideal = total_work * C2 / 2 / nsimd  # every SIMD busy at the two-wave rate
    return {"span_ms": round(ms(span), 2), "ideal_ms": round(ms(ideal), 2),
            "simd_idle": round(idle, 4),
            "simd_end_pct": [round(ms(x), 2) for x in np.percentile(simd_end, [0, 10, 50, 90, 100])],
            "wave_end_pct": [round(ms(x), 2) for x in np.percentile(wave_end, [0, 10, 50, 90, 100])]}


if __name__ == "__main__":
    sizes = c2_segments(int(sys.argv[1]) if len(sys.argv) > 1 else 32768)
    print("segments", len(sizes), "blocks", int(((sizes + 127) // 128).sum()))
    print("lpt prio 8192:", simulate(sizes))
    print("lpt no prio:", simulate(sizes, prio_T=0))
