#!/usr/bin/env python3
"""Check that no instruction touches the destination VGPRs of an LDS read before a
``s_waitcnt lgkmcnt`` has retired it.

The scan kernels issue their table lookups as inline-asm ``ds_read`` with hand-counted waits
(cdc_kernels.hip: PFS_ROLL64G / PFS_ROLL64P).  The compiler believes an asm output is ready
at once, so under register pressure it may copy or spill an in-flight destination before the
wait: a silent race (stale table entries, wrong cuts that change from run to run).  This
walks each function of the device assembly in order, keeps the LDS ops in flight (LDS
returns in issue order; SMEM would break the count, so any s_load makes the check demand
lgkmcnt(0) before its use) and flags a read or write of an in-flight destination register
of a read issued from inline asm (between ;;#ASMSTART and ;;#ASMEND).  The compiler's own
LDS reads count in lgkmcnt like any other, but their registers are never flagged: the
compiler tracks those itself (SIInsertWaitcnts), and the walk is linear in text order, so
out-of-line blocks the compiler places after a read (reached from elsewhere) would otherwise
look like uses of its destination.  A snippet without ASMSTART markers (the self-test) is
treated as asm throughout.

usage: lgkm_hazard_check.py FILE.s [function-substring ...]   (exit 1 on a hazard)
"""
import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def check_function(name, lines):
    inflight = []  # [(dest regs, line no, text)] in issue order (dest empty: count only)
    hazards = []
    has_markers = any(";;#ASMSTART" in raw for _, raw in lines)
    in_asm = not has_markers
    for no, raw in lines:
        if has_markers and ";;#ASMSTART" in raw:
            in_asm = True
            continue
        if has_markers and ";;#ASMEND" in raw:
            in_asm = False
            continue
        line = raw.split(";")[0].strip()
        if not line or line.endswith(":") or line.startswith("."):
            continue
        if line.startswith("s_waitcnt"):
            m = re.search(r"lgkmcnt\((\d+)\)", line)
            if m:
                keep = int(m.group(1))
                while len(inflight) > keep:
                    inflight.pop(0)
            continue
        if line.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
            # control flow: the check is linear, so demand a drained counter at branches the
            # compiler emits (it waits before them itself when it must)
            continue
        op, _, args = line.partition(" ")
        touched = regs(args)
        for dest, at, text in inflight:
            both = dest & touched
            if both:
                hazards.append((no, raw.strip(), at, text, sorted(both)))
        if op.startswith("ds_read") or op.startswith("ds_load"):
            dst = args.split(",")[0]
            inflight.append((regs(dst) if in_asm else set(), no, raw.strip()))
        elif op.startswith(("ds_write", "ds_store", "ds_bpermute", "ds_swizzle", "ds_add",
                            "s_load", "s_buffer_load", "ds_")):
            # an LDS/SMEM op without a tracked destination still counts in lgkmcnt
            d = regs(args.split(",")[0]) if op.startswith(("ds_bpermute", "ds_swizzle")) else set()
            inflight.append((d, no, raw.strip()))
    return hazards


def main():
    path = sys.argv[1]
    want = sys.argv[2:]
    text = open(path).read().split("\n")
    funcs, cur, body = [], None, []
    for no, line in enumerate(text, 1):
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith(".L"):
            if cur:
                funcs.append((cur, body))
            cur, body = m.group(1), []
            continue
        if cur:
            body.append((no, line))
    if cur:
        funcs.append((cur, body))
    bad = 0
    for name, body in funcs:
        if want and not any(w in name for w in want):
            continue
        hz = check_function(name, body)
        print("%-90s %d hazard(s)" % (name[:90], len(hz)))
        for h in hz[:10]:
            print("   line %d: %s  <- in flight since line %d: %s  regs %s" % h)
        bad += len(hz)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
