"""A CPU model of the scan's cut skipping (cdc_kernels.hip scan_unit_plan / record_block /
scan_unit_report), checked under random unit timings and stale reads.

The GPU tests compare the kernel's results with the oracle at a few timings (one, three and
all scan workgroups).  This model replays the same rules -- rank-ordered dispatch, per-file
rank slots holding a done bit and a unit's lowest candidate, the replay of the selection
over them -- with units that start and finish in random order, slots read at random times,
and a reader that sees a random subset of the slots' updates (each slot self-consistent).
The property: selecting over the candidates the scan still found gives exactly the cuts of
selecting over every candidate (writer.go:163-189 through oracle.chunker's select rule).

Candidate positions are drawn directly (the replay depends on where candidates are, not on
the rolling hash); the geometry is scaled down (unit U, step U / 32, min > U) so thousands
of timings run in seconds.  Test infrastructure only: nothing here runs on the product path.
"""
import numpy as np
import pytest

U = 1024          # work unit (the kernel's kScanUnit, scaled down)
STEP = U // 32    # skip granularity (kUnitStep)
SLOTS = 64        # rank slots per file (kRankSlots)


def select_cuts(cands, fs, fe, mn, mx):
    """select_file: the cut positions of one file from a sorted candidate array."""
    cuts, s = [], fs
    while True:
        lo = s + mn - 1
        if lo >= fe:
            break
        hi = s + mx - 1
        limit = min(hi, fe - 1)
        k = np.searchsorted(cands, lo)
        c = int(cands[k]) if k < len(cands) and cands[k] <= limit else None
        if c is None:
            if hi <= fe - 1:
                c = hi
            else:
                break
        cuts.append(c)
        s = c + 1
    return cuts


def plan_units(offs, mn):
    """scan_skip_kernel: per unit its static skip (steps), tracked file and rank."""
    n = int(offs[-1])
    nfiles = len(offs) - 1
    kall = U // STEP
    units = []
    for u in range((n + U - 1) // U):
        ub, ue = u * U, min((u + 1) * U, n)
        f = int(np.searchsorted(offs, ub, side="right") - 1)
        s, tf, rank = 0, None, 0  # the kernel starts from "scan whole" (a crowded unit)
        for g in range(f, f + 64):
            if g >= nfiles or offs[g] >= ue:
                s = kall
                break
            ls, fe = int(offs[g]) + mn - 1, int(offs[g + 1])
            if ls < fe:
                first = max(ls, ub)
                s = (first - ub) // STEP if first < ue else kall
                tf, rank = g, ub // U - ls // U
                break
        if tf is None:
            s = kall  # plan mode: a crowded unit holds no eligible position, takes no slot
        if s < kall and ub + s * STEP < ue:
            units.append((u, tf, rank, s))
    units.sort(key=lambda t: (min(t[2], 63), t[0]))
    return units


def replay(view, f, rank, offs, mn, mx):
    """scan_unit_plan's replay: the first eligible position after the last settled cut
    before this unit (0: none).  view[q] = (done, lowest candidate or None) for rank q."""
    fs, fe = int(offs[f]), int(offs[f + 1])
    e = fs + mn - 1
    u0 = e // U
    rlim = min(rank, SLOTS)
    lo, hi, d = e, fs + mx - 1, 0
    for _ in range(SLOTS):
        qlo = lo // U - u0
        if qlo >= rlim:
            break
        qc = next((q for q in range(qlo, SLOTS) if view[q][1] is not None), 64)
        c = view[qc][1] if qc < 64 else None
        if qc == qlo and c < lo:
            break  # lo's own unit: a later candidate may follow its lowest
        if c is not None and c <= hi and c < fe:
            cut, qneed = c, qc
        else:
            if hi >= fe:
                break
            cut, qneed = hi, hi // U - u0
        if qneed >= rlim or not all(view[q][0] for q in range(qlo, qneed + 1)):
            break
        d = cut + mn
        lo, hi = d, cut + mx
    return d


def simulate(offs, cands, mn, mx, rng, waves, stale):
    n = int(offs[-1])
    units = plan_units(offs, mn)
    nfiles = len(offs) - 1
    # slot state per file and rank: a history of (time, done, lowest candidate) updates
    hist = {}
    found = []
    t_free = [0.0] * waves
    for (u, f, rank, s) in units:
        w = int(np.argmin(t_free))
        start = t_free[w] + rng.random() * 0.2
        ub, ue = u * U, min((u + 1) * U, n)
        if rank >= 1:
            view = []
            for q in range(SLOTS):
                ups = [x for x in hist.get((f, q), []) if x[0] <= start]
                if ups and stale and rng.random() < stale:
                    ups = ups[:rng.integers(0, len(ups) + 1)]  # an older, self-consistent value
                done = bool(ups) and ups[-1][1]
                low = min((x[2] for x in ups if x[2] is not None), default=None)
                view.append((done, low))
            d = replay(view, f, rank, offs, mn, mx)
            if d > ub:
                s = max(s, min((d - ub) // STEP, U // STEP))
        a = ub + s * STEP
        dur = 0.5 + rng.random()
        mine = cands[(cands >= a) & (cands < ue)]
        found.append(mine)
        if rank < SLOTS:
            ups = hist.setdefault((f, rank), [])
            for k, c in enumerate(mine):  # candidates reported as the unit meets them
                ups.append((start + dur * (k + 1) / (len(mine) + 1), False, int(c)))
            ups.append((start + dur, True, None))
            ups.sort(key=lambda x: x[0])
        t_free[w] = start + dur
    got = np.unique(np.concatenate(found)) if found else np.zeros(0, np.int64)
    return got, nfiles


@pytest.mark.parametrize("avg,mn,mx", [(300, 1100, 4000), (2500, 1100, 3000),
                                       (150, 2200, 9000), (10**9, 1100, 2500)])
def test_replay_never_hides_a_cut(avg, mn, mx):
    rng = np.random.default_rng(avg + mn)
    for trial in range(6):
        lens = rng.integers(0, 12 * U, 40)
        lens[rng.integers(0, 40, 4)] = rng.integers(30 * U, 70 * U, 4)  # long files: 64+ ranks
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        n = int(offs[-1])
        cands = np.unique(rng.integers(0, n, max(1, n // avg))) if avg < n else np.zeros(0, np.int64)
        want = [select_cuts(cands, int(offs[f]), int(offs[f + 1]), mn, mx)
                for f in range(len(offs) - 1)]
        for waves, stale in ((1, 0.0), (3, 0.3), (12, 0.0), (12, 0.7)):
            got, nfiles = simulate(offs, cands, mn, mx, rng, waves, stale)
            for f in range(nfiles):
                assert select_cuts(got, int(offs[f]), int(offs[f + 1]), mn, mx) == want[f], \
                    (trial, waves, stale, f)


def test_crowded_units_take_no_slot_and_hide_no_cut():
    """Units crowded with more than 64 sub-min files: with min - 1 >= one unit
    they hold no eligible position, so they take no dispatch slot (the kernel's slot count and
    the slots it fills must agree), and the cuts of the long files around them are unchanged."""
    rng = np.random.default_rng(11)
    mn, mx = 1100, 4000
    lens = np.concatenate([[30 * U], np.full(400, 9), [25 * U], np.full(200, 13), [40 * U]])
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    units = plan_units(offs, mn)
    assert all(tf is not None for (_, tf, _, _) in units)
    crowded = [u for u in range(int(offs[-1]) // U)
               if np.count_nonzero((offs[:-1] >= u * U) & (offs[:-1] < (u + 1) * U)) > 64]
    assert crowded, "the layout must crowd at least one unit"
    n = int(offs[-1])
    cands = np.unique(rng.integers(0, n, n // 300))
    want = [select_cuts(cands, int(offs[f]), int(offs[f + 1]), mn, mx)
            for f in range(len(offs) - 1)]
    for waves, stale in ((1, 0.0), (12, 0.5)):
        got, nfiles = simulate(offs, cands, mn, mx, rng, waves, stale)
        for f in range(nfiles):
            assert select_cuts(got, int(offs[f]), int(offs[f + 1]), mn, mx) == want[f]


def test_replay_skips_something_when_ranks_finish_in_order():
    """With one wave the earlier ranks have always reported: files carry chains of cuts and
    the scan must skip past them (else the model tests nothing)."""
    rng = np.random.default_rng(5)
    lens = np.full(30, 20 * U)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    n = int(offs[-1])
    cands = np.unique(rng.integers(0, n, n // 400))
    got, _ = simulate(offs, cands, 1100, 4000, rng, 1, 0.0)
    assert len(got) < len(cands[cands >= 1100 - 1])
