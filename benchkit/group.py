"""Device group (--path group): one process, one library context per member device, the
step's files dealt over the members (pfscdc_deal), scanned and hashed concurrently and the
chunk-ref index gathered peer to peer onto the first member's device (pfscdc_group_scan_resident,
include/pfscdc.h).  This is what a cgo pachd calls to use a node's GPUs.  --members lists the
member devices (default: every visible device once; on a one-GPU box "0,0,0,0" puts four
contexts on the one GPU).  Beside the group's line: one context alone over the same files, and
the gathered index's digest against it."""
import hashlib

from .common import GIB, med
from .harness import Harness


def bench_group(args, ctx):
    np, torch = ctx["np"], ctx["torch"]
    from pfs_amd.group import DeviceGroup

    H = Harness(ctx)
    if ctx["world"] > 1:
        raise SystemExit("--path group is one process driving several devices (no ranks)")
    ndev = torch.cuda.device_count()
    members = [int(x) for x in args.members.split(",")] if args.members else list(range(ndev))
    batches = args.group if args.group > 0 else 8
    nfiles = args.files * batches
    offs = np.arange(nfiles + 1, dtype=np.uint64) * np.uint64(args.file_bytes)
    seed = 0xC2 if args.seed < 0 else args.seed
    total = int(offs[-1])

    def run_group(devs, steps, warmup):
        g = DeviceGroup(devs, ctx["params"])
        parts = g.fill_synthetic_resident(offs, seed)
        for _ in range(warmup):
            g.scan_resident(parts, offs)
        tm, last = [], {}

        def run(k):
            for _ in range(k):
                last["r"] = g.scan_resident(parts, offs)
                tm.append(g.timings())

        elapsed = H.timed(run, steps)
        r = last["r"]
        digest = hashlib.blake2b(r.segments.tobytes() + r.file_begin.tobytes(),
                                 digest_size=16).hexdigest()
        out = {"elapsed": elapsed, "digest": digest, "segments": int(len(r.segments)),
               "part_begin": [int(x) for x in g.part_begin()],
               "member_ms": [med([t["member_ms"][k] for t in tm]) for k in range(len(devs))],
               "gather_ms": med([t["gather_ms"] for t in tm]),
               "gather_bytes": tm[-1]["gather_bytes"] if tm else 0}
        g.close()
        del parts
        torch.cuda.empty_cache()
        return out

    grp = run_group(members, args.steps, args.warmup)
    one = run_group([members[0]], args.steps, args.warmup)
    info = {"workload": "configs[1] batches of %d x %d B, %d per step, resident on the members"
                        % (args.files, args.file_bytes, batches),
            "path": "group (pfscdc_group_scan_resident: dealt scan + hash, peer-to-peer gather)",
            "members": members, "part_begin": grp["part_begin"],
            "parallelism": "%d contexts in one process over devices %s" % (
                len(members), sorted(set(members)))}
    line = H.line("GiB/s device-resident CDC rolling-hash + chunk content-hash, device group",
                  total, args.steps, args.warmup, grp["elapsed"], "strong", info,
                  member_ms=grp["member_ms"], gather_ms=grp["gather_ms"],
                  gather_bytes=grp["gather_bytes"], segments=grp["segments"],
                  one_context={"value": round(total * args.steps / one["elapsed"] / GIB, 3),
                               "unit": "GiB/s", "ms_per_step": round(one["elapsed"] * 1e3 /
                                                                     max(args.steps, 1), 3),
                               "device": members[0]},
                  parity={"index_digest": grp["digest"],
                          "equals_one_context": grp["digest"] == one["digest"]})
    H.emit(line)
