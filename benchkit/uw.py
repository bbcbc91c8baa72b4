"""Host-fed pachd write path (--path uw): the first --uw-bytes of the commit's files (host
memory) Put through the UnorderedWriter (pfs_amd.fileset over pfscdc_uw_*): buffering,
1e9-byte filesets, GPU chunk writers with Ref ids, index writers.  N > 1: whole serialized
filesets per rank (each rank its own UnorderedWriter over its pieces, the re-Added
continuation of a split file Put with append); the filesets (SizeBytes, root indexes) are
gathered: the same list as one writer's.  Reference: fileset/unordered_writer.go:45-179."""
import hashlib
import time

from .common import Work, c4_sizes, fill, host_memcpy_rate, workload
from .harness import Harness


def bench_uw(args, ctx):
    np, torch, pd = ctx["np"], ctx["torch"], ctx["pd"]
    world, rank, dev, cdev, params = ctx["world"], ctx["rank"], ctx["dev"], ctx["cdev"], ctx["params"]
    from pfs_amd import _lib
    from pfs_amd import fileset as pf
    from pfs_amd.cdc import Chunker

    H = Harness(ctx)
    base = workload(args, 1, 0) if args.config in ("c2", "c3") else None
    if base is None:
        sizes = c4_sizes()
        seed = (0xC4 if args.config == "c4" else 0xC5) if args.seed < 0 else args.seed
        mode = workload(args, 1, 0).mode if args.config == "c5" else 0
    else:
        sizes, seed, mode = base.sizes, base.seed, base.mode
    offs = np.zeros(len(sizes) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(np.asarray(sizes, dtype=np.uint64))
    nf = max(1, int(np.searchsorted(offs, min(args.uw_bytes, int(offs[-1])), side="right")) - 1)
    lay = pd.commit_layout(sizes[:nf], args.mem_threshold)
    fs = pd.shard_filesets(lay, world)[rank]
    p0, p1 = pd.rank_pieces(lay, fs)
    pieces = Work(lay.size[p0:p1], lay.file[p0:p1], lay.start[p0:p1], seed, mode, {}, "strong")
    nbytes = pieces.total
    gen = Chunker(params, device=ctx["local"])
    t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
    fill(gen, t, pieces)
    host = t[:nbytes].cpu().numpy()
    gen.close()
    del t
    torch.cuda.empty_cache()
    views = {}  # (file, start) -> the piece's bytes in host memory
    for i in range(p0, p1):
        o = int(pieces.offs[i - p0])
        views[(int(lay.file[i]), int(lay.start[i]))] = memoryview(host[o:o + int(lay.size[i])])
    if args.uw_workers > 0:
        _lib.set_knob("PFSCDC_UW_WORKERS", args.uw_workers)
    if args.uw_group > 0:
        _lib.set_knob("PFSCDC_UW_INFLIGHT", args.uw_group)
    members = [int(x) for x in args.members.split(",")] if args.members else None
    if members and world > 1:
        raise SystemExit("--members (a device group in one process) with --gpus > 1")
    st = pf.Storage(ctx["local"], params, args.mem_threshold, devices=members)
    last = {}

    def step():
        t0 = time.perf_counter()
        w = st.new_unordered_writer()
        create_ms = (time.perf_counter() - t0) * 1e3
        prims = pd.put_rank_filesets(w, lay, fs, lambda f: "/%016d" % f,
                                     lambda f, s, n: views[(f, s)])
        tm = w.timings()
        tm["writer_create"] = create_ms
        nch = sum(1 for fsv in w.events for e in fsv if e[0] == "chunk" and e[1] == -1)
        w.release()  # its data context goes back to the Storage for the next commit
        return prims, tm, nch

    stages = {}

    def run(k):
        for _ in range(k):
            prims, tm, nchunks = step()
            last.update(prims=prims, nchunks=nchunks)
            for key, v in tm.items():
                stages[key] = stages.get(key, 0.0) + v / max(args.steps, 1)

    for _ in range(args.warmup):
        step()
    elapsed = H.timed(run, args.steps)
    bytes_step = H.sum_over_ranks(nbytes)
    prims = last["prims"]
    gathered = pd.gather_primitives(prims, device=cdev) if world > 1 else \
        [(p.additive, p.deletive, p.size_bytes) for p in prims]
    info = {"workload": "the first %d files (%d B) of %s, Put from host memory" % (
                nf, int(offs[nf]), args.config),
            "path": "uw (host-fed UnorderedWriter -> fileset.Writer -> index.Writer)",
            "bytes_this_rank": nbytes, "mem_threshold": args.mem_threshold,
            "filesets": lay.nfilesets, "filesets_this_rank": len(prims),
            "data_chunks_this_rank": last["nchunks"], "gpu_max_hw_queues": ctx["hwq"],
            "parallelism": "fileset-sharded x%d, gather of the fileset roots" % world
            if world > 1 else ("device group over %s (pfscdc_uw_create_group)" % members
                               if members else "single GPU")}
    out = H.line("GiB/s host-fed pachd write path (Put -> filesets with chunk Refs and "
                 "multilevel indexes)", bytes_step, args.steps, args.warmup, elapsed, "strong",
                 info, data="synthetic bytes in host memory",
                 commit_filesets_digest=hashlib.blake2b(
                     b"".join(pd.encode_primitive(*g) for g in gathered),
                     digest_size=16).hexdigest(),
                 note="a step: the Puts (one host copy into the fileset arenas) and the grouped "
                      "GPU write of every fileset plus the indexes, then Close",
                 stages_ms={k: round(v, 2) for k, v in stages.items()},
                 stages_note="per step; put_copy on the Put thread, the rest summed over the "
                             "group writes (a background thread per group writer, %d writer(s), "
                             "each on its own ctx), so they overlap the Puts and each other "
                             "(pfscdc_uw_timings)" % _lib.get_knob("PFSCDC_UW_WORKERS"))
    if stages.get("put_copy"):
        out["put_copy_gb_s"] = round(nbytes / (stages["put_copy"] * 1e-3) / 1e9, 2)
        out["host_memcpy_gb_s"] = host_memcpy_rate(torch, min(nbytes, 4 << 30))
    H.emit(out)
    H.close()
