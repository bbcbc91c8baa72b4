"""pachd data plane on device-resident files (--path commit): pieces / filesets
(commit_layout), CDC + DataRef hashes (one scan of all pieces), chunk formation per fileset
stream (pfscdc_form_chunks), chunk.Create of every formed chunk (pfscdc_commit_refs: DataRef
and content hashes in one launch, dek, ChaCha20 + BLAKE2b of the ciphertext).

N > 1: whole serialized filesets per rank (a fresh chunk.Writer per fileset, so chunks never
span ranks); each rank forms its chunks and Refs, and the chunk records (offset in the commit
stream, size, Ref.Id, Ref.Dek) are gathered to rank 0: the same list as N = 1.

With --inflight S > 1, S contexts (S HIP streams) each run every S-th step from their own host
thread, so one step's chunk.Create tail (the serial BLAKE2b chains of its largest chunks:
content hash, then Ref.Id) overlaps the next step's scan and hashes.  The steps read the same
device buffer (the same files committed again; the library only reads it)."""
import hashlib
import threading
import time

from .common import HBM_PEAK_GBS, Work, fill, workload
from .harness import Harness, plan_steps


def bench_commit(args, ctx):
    np, torch, pd = ctx["np"], ctx["torch"], ctx["pd"]
    world, rank, dev, cdev, params = ctx["world"], ctx["rank"], ctx["dev"], ctx["cdev"], ctx["params"]
    from pfs_amd.cdc import Chunker

    H = Harness(ctx)
    if args.config not in ("c4", "c5"):
        args.group = 1
    # c4/c5: --group G commits per step per GPU (auto: >= MIN_CHAINS BLAKE2b chains, as the
    # put path), each copy the same layout over its own files
    work = workload(args, world, rank) if args.config in ("c4", "c5") else None
    if work is None:  # c2/c3 files committed as one commit: pieces per fileset
        base = workload(args, 1, 0)
        lay = pd.commit_layout(base.sizes, args.mem_threshold)
        fs = pd.shard_filesets(lay, world)[rank]
        p0, p1 = pd.rank_pieces(lay, fs)
        ids = base.ids[lay.file[p0:p1]]
        starts = base.starts[lay.file[p0:p1]] + lay.start[p0:p1]
        work = Work(lay.size[p0:p1], ids, starts, base.seed, base.mode, base.info, "strong",
                    gbase=p0)
        work.layout, work.fs_range = lay, fs
    lay, fs = work.layout, work.fs_range
    p0 = work.gbase
    G, per_copy = work.group, work.per_copy
    s1 = (lay.fileset_begin[fs[0]:fs[1] + 1] - p0).astype(np.uint32)  # one copy's streams
    streams = np.concatenate([s1[:1]] + [s1[1:] + np.uint32(g * per_copy) for g in range(G)]) \
        if len(s1) else s1
    total = work.total
    total0 = int(work.offs[per_copy])  # copy 0: the commit itself
    S = args.inflight if args.inflight > 0 else 1
    steps, warmup, steps_note = plan_steps(args.steps, args.warmup, S)
    data = torch.empty(total, dtype=torch.uint8, device=dev)
    chunkers = [Chunker(params, device=ctx["local"]) for _ in range(S)]
    fused = args.commit_hash == "fused"
    # the ciphertext over the plaintext (PFSCDC_OPT_CTEXT_IN_PLACE) when a ciphertext copy of
    # the step would not fit beside it: the split Ref.Id pass without a second buffer
    _, hbm = torch.cuda.mem_get_info(dev)
    in_place = fused and not args.no_create and (
        args.in_place == 1 or (args.in_place < 0 and 2 * total + (16 << 30) > hbm))
    for ch in chunkers:  # the DataRef hashes join the chunk content hashes (pfscdc_commit_refs)
        ch.set_cuts_only(fused)
        ch.set_ctext_in_place(in_place)
    fill(chunkers[0], data, work)
    poffs = work.offs
    gbyte = int(lay.offsets()[p0])  # this rank's first byte in the commit stream
    keys = ("scan", "hash", "total", "create", "create_content_hash", "create_ref_id",
            "host_form_ms")
    accs = [dict.fromkeys(keys, 0.0) for _ in range(S)]
    lasts = [{} for _ in range(S)]

    def step(k, record):
        chunker, acc = chunkers[k], accs[k]
        res = chunker.scan(data, poffs)
        if record:
            t = chunker.timings()
            for name in ("scan", "hash", "total"):
                acc[name] += t[name]
        h0 = time.perf_counter()
        coffs, hashes, known = chunker.form_chunks(streams)
        if record:
            acc["host_form_ms"] += (time.perf_counter() - h0) * 1e3
        if fused:
            refs, chash, seghash = chunker.commit_refs(data, coffs, known,
                                                       create=not args.no_create)
            res.segments["hash"] = seghash
        else:
            refs, chash = chunker.create_refs(data, coffs, hashes, known)
        if record:
            acc["create"] += chunker.last_create_ms()
            ct = chunker.last_create_timings()
            acc["create_content_hash"] += ct["content_hash"]
            acc["create_ref_id"] += ct["ref_id"]
        lasts[k].update(res=res, coffs=coffs, known=known, refs=refs,
                        chash=chash if fused else None)

    errors = []

    def worker(k, nsteps, record):
        try:
            for _ in range(nsteps):
                step(k, record)
        except BaseException as e:  # re-raised on the main thread
            errors.append(e)

    def run(nsteps, record=True):
        """nsteps steps, step i on context i % S; one host thread per context."""
        counts = [len(range(k, nsteps, S)) for k in range(S)]
        if S == 1:
            worker(0, counts[0], record)
        else:
            ts = [threading.Thread(target=worker, args=(k, counts[k], record))
                  for k in range(S) if counts[k]]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        if errors:
            raise errors[0]

    for k in range(S):  # every context warms up (buffers sized) before the timed region
        worker(k, max(warmup // S, 1) if S > 1 else warmup, False)
    if errors:
        raise errors[0]
    elapsed = H.timed(run, steps)
    bytes_step = H.sum_over_ranks(total)
    K = max(steps, 1)
    avg = {name: sum(a[name] for a in accs) / K for name in keys}
    if in_place:
        # the timed steps each read the previous step's ciphertext (pseudo-random bytes, like
        # the synthetic input); the digests and the parity check come from one more step over
        # the synthetic commit itself, after the timed region
        torch.cuda.synchronize()
        fill(chunkers[0], data, work)
        step(0, False)
    last = lasts[0]
    coffs, known = last["coffs"], last["known"]
    nch_all = len(coffs) - 1
    # copy 0 (the commit itself) is what the digests and the gathered list cover: equal at
    # every N and G
    nch = int(np.searchsorted(coffs, np.uint64(total0), side="left")) if G > 1 else nch_all
    # the commit's chunk list: (offset in the commit stream, size, Ref.Id, Ref.Dek) per chunk
    # (with --no-create: the content hash in place of Ref.Id, Dek zero)
    cdt = np.dtype([("offset", "<u8"), ("size", "<u8"), ("id", "u1", (32,)), ("dek", "u1", (32,))])
    crec = np.zeros(nch, dtype=cdt)
    crec["offset"] = coffs[:nch] + np.uint64(gbyte)
    crec["size"] = np.diff(coffs[:nch + 1])
    if last.get("refs") is not None:
        crec["id"] = last["refs"]["id"][:nch]
        crec["dek"] = last["refs"]["dek"][:nch]
    else:
        crec["id"] = last["chash"][:nch]
    chunks = pd.gather_records_to_root(crec, device=cdev) if world > 1 else crec
    if chunks is None:  # not rank 0: nothing gathered here, nothing printed
        chunks = crec[:0]
    segs0 = last["res"].segments
    segs0 = segs0[segs0["file"] < per_copy]
    dr_hashes = np.ascontiguousarray(segs0["hash"]).view(np.dtype((np.void, 32))).reshape(-1)
    if world > 1:  # the commit's DataRef hashes in commit order: equal at every N
        dr_hashes = pd.gather_records_to_root(dr_hashes, device=cdev)
        if dr_hashes is None:
            dr_hashes = np.zeros(0, dtype=np.dtype((np.void, 32)))
    info = dict(work.info)
    info.update({"path": "commit (UnorderedWriter filesets -> chunk.Writer streams -> "
                         "chunk.Create)", "mem_threshold": args.mem_threshold,
                 "filesets_this_rank": fs[1] - fs[0], "pieces_this_rank": len(work.sizes),
                 "chunks_this_rank": nch, "chunks_per_commit": int(len(chunks)),
                 "multi_dataref_chunks": int(nch - int(known[:nch].sum())),
                 "commits_per_step": G, "chunks_per_step": nch_all,
                 "ciphertext_in_place": in_place,
                 "chunk_create": not args.no_create,
                 "commit_hash": args.commit_hash,
                 "steps_in_flight": S, "gpu_max_hw_queues": ctx["hwq"],
                 "parallelism": "fileset-sharded x%d, chunk records gathered to rank 0" % world
                 if world > 1 else "single GPU"})
    ms = avg["create"]
    ach = total / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    metric = ("GiB/s device-resident pachd commit data plane (CDC + DataRef hashes + "
              "chunk formation + chunk.Create Ref.Id)") if not args.no_create else (
              "GiB/s device-resident CDC + every BLAKE2b of Writer.processChunk (DataRef hashes "
              "+ chunk content hashes, writer.go:240,301-312) + chunk formation")
    out = H.line(metric, bytes_step, steps, warmup, elapsed,
                 work.scaling if G > 1 else "strong", info,
                 kernel_ms={name: round(v, 4) for name, v in avg.items()},
                 commit_chunks_digest=hashlib.blake2b(chunks.tobytes(), digest_size=16).hexdigest(),
                 dataref_hashes_digest=hashlib.blake2b(dr_hashes.tobytes(),
                                                       digest_size=16).hexdigest(),
                 roofline={"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                           "bytes_per_launch": total, "avg_launch_ms": round(ms, 4),
                           "kernel": "chunk.Create batch (content hash + dek + ChaCha20/BLAKE2b)"
                           if not args.no_create else
                           "one BLAKE2b launch over every segment and multi-DataRef chunk"})
    if steps_note:
        out["steps_requested"], out["warmup_requested"] = args.steps, args.warmup
        out["steps_rule"] = steps_note
    if S > 1:
        out["note"] = ("kernel_ms are per step on its own stream; with %d steps in flight they "
                       "overlap, so ms_per_step < their sum" % S)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if in_place:  # the buffer holds the verification step's ciphertext
            fill(chunkers[0], data, work)
        out["parity"] = commit_parity(data, work, streams, last, params, np)
    H.emit(out)
    H.close()
    for ch in chunkers:
        ch.close()


def commit_parity(data, work, streams, last, params, np):
    """The first fileset through the CPU oracle: segments (C restatement), the chunk.Writer
    replay (oracle.chunker), and chunk.Create of a sample of its chunks."""
    from oracle import chunker as och
    from oracle import coracle

    poffs = work.offs
    f1 = int(streams[1])
    nb = int(poffs[f1])
    host = data[:nb].cpu().numpy()
    p = och.Params(params.average_bits, params.seed, params.min_chunk, params.max_chunk)
    segs, begin = coracle.segment_files(host, poffs[:f1 + 1], p, nthreads=16)
    w = och._SegmentReplayWriter(params=p)
    for f in range(f1):
        a = int(poffs[f])
        w.annotate(och.Annotation(data=f))
        w.write_segments(host[a:int(poffs[f + 1])].tobytes(),
                         [(int(s["offset"]), int(s["size"]), bool(s["flags"] & 2))
                          for s in segs[int(begin[f]):int(begin[f + 1])]])
    w.close()
    want = np.concatenate([[0], np.cumsum([len(c.data) for c in w.chunks])]).astype(np.uint64)
    coffs = last["coffs"]
    n = len(want) - 1
    same_cuts = bool(np.array_equal(coffs[:n + 1], want))
    ok = True
    idx = np.unique(np.linspace(0, n - 1, min(8, n)).astype(int))
    if last.get("refs") is None:  # --no-create: the chunk content hashes
        for i in idx:
            ok &= bytes(last["chash"][i]) == hashlib.blake2b(w.chunks[i].data,
                                                             digest_size=32).digest()
        return {"first_fileset_chunk_offsets_equal_oracle": same_cuts, "chunks": n,
                "content_hashes_equal_oracle": bool(ok), "content_hashes_checked": int(len(idx))}
    for i in idx:
        rid, dek = och.create_ref_id(w.chunks[i].data)
        ok &= bytes(last["refs"][i]["id"]) == rid and bytes(last["refs"][i]["dek"]) == dek
    return {"first_fileset_chunk_offsets_equal_oracle": same_cuts, "chunks": n,
            "ref_ids_equal_oracle": bool(ok), "ref_ids_checked": int(len(idx))}
