"""Read a PFSCDC_WAVE_TRACE file (development tool): per hash launch, how the waves, SIMDs and
CUs of the launch drain.  Each record: span[4] (scan begin/end, hash begin/end; s_memrealtime
ticks, 100 MHz) then 32768 x (end tick, HW_ID | XCC_ID << 32, blocks run, shader cycles) per
wave slot."""
import sys

import numpy as np

TICK_MS = 1e-5  # 100 MHz
raw = np.fromfile(sys.argv[1], dtype=np.uint64)
rec = 4 + 4 * 32768
for k in range(len(raw) // rec):
    r = raw[k * rec:(k + 1) * rec]
    hb, he = int(r[2]), int(r[3])
    w = r[4:].reshape(-1, 4)
    w = w[w[:, 0] != 0]
    end = (w[:, 0].astype(np.int64) - hb) * TICK_MS
    hw = w[:, 1]
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = (hw >> 32) & 15
    T = (he - hb) * TICK_MS
    simd_key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    cu_key = simd_key // 4
    def ends(key):
        u, inv = np.unique(key, return_inverse=True)
        m = np.zeros(len(u))
        np.maximum.at(m, inv, end)
        return m
    se_, ce = ends(simd_key), ends(cu_key)
    q = lambda a: " ".join(f"{x:6.2f}" for x in np.percentile(a, [0, 10, 50, 90, 100]))
    print(f"launch {k}: {len(w)} waves, hash span {T:.2f} ms; percentiles 0/10/50/90/100 of end (ms):")
    print(f"  waves  {q(end)}\n  SIMDs  {q(se_)}  ({len(se_)} SIMDs)\n  CUs    {q(ce)}  ({len(ce)} CUs)")
    steps = w[:, 2].astype(np.float64)
    print(f"  blocks run per wave: {q(steps)}; sum {steps.sum():.4g} wave-blocks "
          f"(x16 quads = {steps.sum() * 16:.4g} quad-block slots)")
    print(f"  SIMD-time idle after the SIMD's last wave: {np.sum(T - se_) / (len(se_) * T) * 100:.2f}%"
          f"; CU-time idle after the CU's last wave: {np.sum(T - ce) / (len(ce) * T) * 100:.2f}%")
    # per XCD: when its SIMDs end (a slow XCD bounds a launch whose waves hold equal work)
    ukey, inv = np.unique(simd_key, return_inverse=True)
    m = np.zeros(len(ukey))
    np.maximum.at(m, inv, end)
    sx = (ukey // (8 * 2 * 16 * 4)).astype(int)
    print("  per XCD: mean / max SIMD end (ms): " + "  ".join(
        f"{x}: {m[sx == x].mean():.2f}/{m[sx == x].max():.2f}" for x in np.unique(sx)))
    cyc = w[:, 3].astype(np.float64)
    if cyc.any():  # each wave's lifetime in shader cycles over its wall time: its clock
        mhz = cyc / np.maximum(end, 1e-3) / 1e3
        wx = ((simd_key // (8 * 2 * 16 * 4)).astype(int))
        print("  per XCD: mean wave clock (MHz): " + "  ".join(
            f"{x}: {mhz[wx == x].mean():.0f}" for x in np.unique(wx)))
