#!/usr/bin/env python3
"""Timeline of one step from a rocprofv3 --kernel-trace csv: every kernel launched between
the k-th-from-last launch of the step's first kernel and the next one, with start/end relative
to the step start, its queue, and how much of the step at least one kernel was running.

usage: kernel_timeline.py KERNEL_TRACE.csv [first-kernel-substring=cdc_scan_kernel] [k=2]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "cdc_scan_kernel"
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    rows = list(csv.DictReader(open(path)))
    name_key = next(c for c in rows[0] if c.lower() in ("kernel_name", "kernelname"))
    s_key = next(c for c in rows[0] if "start" in c.lower())
    e_key = next(c for c in rows[0] if "end" in c.lower())
    q_key = next((c for c in rows[0] if "queue" in c.lower()), None)
    ks = sorted(((int(r[s_key]), int(r[e_key]), r[name_key], r.get(q_key, "")) for r in rows))
    starts = [s for s, e, n, q in ks if first in n]
    if len(starts) < k:
        print("only", len(starts), "launches of", first)
        return 1
    t0 = starts[-k]
    t1 = starts[-k + 1] if k > 1 else max(e for s, e, n, q in ks)
    step = [(s, e, n, q) for s, e, n, q in ks if t0 <= s < t1]
    end = max(e for s, e, n, q in step)
    print("step: %d kernels, %.2f ms from the first %s to the last kernel end" %
          (len(step), (end - t0) / 1e6, first))
    for s, e, n, q in step:
        short = n.split("(")[0].replace("void pfscdc::", "")[:60]
        print("  %9.2f %9.2f %8.2f ms  q%-4s %s" % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6, q, short))
    # union of busy intervals
    busy, cur_s, cur_e = 0, None, None
    for s, e, n, q in sorted(step):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print("busy (some kernel running): %.2f of %.2f ms" % (busy / 1e6, (end - t0) / 1e6))
    return 0


if __name__ == "__main__":
    sys.exit(main())
