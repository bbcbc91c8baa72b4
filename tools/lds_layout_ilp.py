"""Is there a bank-conflict-free LDS layout for the quad kernel's message reads?
(development tool).

A ds_read_b64 lane group is 32 lanes = 8 quads; in each (round, step) every quad's 4 lanes
read the same 4 message words (one per lane), so a read is conflict-free iff the 8 x 4
(quad, word) cells land on 32 distinct bank pairs.  The placement f(quad, word) -> bank pair
may differ per quad.  This poses "every one of the 40 distinct word groups is a bijection"
as a 0/1 program for HiGHS (scipy.optimize.milp) and reports feasibility (it is not)."""
import numpy as np
from scipy.optimize import Bounds, LinearConstraint, milp

SIGMA = [
    [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15],
    [14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3],
    [11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4],
    [7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8],
    [9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13],
    [2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9],
    [12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11],
    [13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10],
    [6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5],
    [10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0],
]
# the word set read by one instruction: x0 = s[2j], x1 = s[2j+1] (column step) and
# s[8+2i], s[9+2i] (diagonal step) over the quad's 4 lanes; the set does not depend on
# which lane runs which diagonal
GROUPS = []
for s in SIGMA:
    for b in (0, 1, 8, 9):
        GROUPS.append([s[b], s[b + 2], s[b + 4], s[b + 6]])

NQ, NW, NB = 8, 16, 32


def var(q, w, b):
    return (q * NW + w) * NB + b


def main():
    n = NQ * NW * NB
    rows, lo, hi = [], [], []
    for q in range(NQ):
        for w in range(NW):
            r = np.zeros(n)
            r[[var(q, w, b) for b in range(NB)]] = 1
            rows.append(r), lo.append(1), hi.append(1)
    for g in GROUPS:
        for b in range(NB):
            r = np.zeros(n)
            r[[var(q, w, b) for q in range(NQ) for w in g]] = 1
            rows.append(r), lo.append(1), hi.append(1)
    res = milp(c=np.zeros(n), constraints=LinearConstraint(np.array(rows), lo, hi),
               integrality=np.ones(n), bounds=Bounds(0, 1), options={"time_limit": 900})
    print(f"{len(GROUPS)} word groups; conflict-free per-quad layout: "
          f"{'exists' if res.status == 0 else 'none'} ({res.message})")


if __name__ == "__main__":
    main()
