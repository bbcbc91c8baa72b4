"""The ingest path (the headline): CDC scan + cut selection + BLAKE2b of every segment over
device-resident synthetic files, for configs[1] (c2), configs[2] at N = 1 (c3), configs[3]
(c4) and configs[4] (c5).  N > 1: every rank its own share (c2: its own files, weak scaling;
c4/c5: whole serialized filesets), the chunk-ref index gathered to rank 0 every step."""
import hashlib
import statistics
import time

from . import parity as par
from .common import (GIB, HBM_PEAK_GBS, LITERAL_INFLIGHT, METRIC, SIMDS, VALU_PEAK_GIPS,
                     C3_INFLIGHT, C3_SCAN_GRID, fill, hit_rate, load_traffic, med, workload)
from .harness import Harness, plan_steps, steady_state


def inflight_for(args) -> int:
    """Steps in flight.  One at a time by default, so every kernel launch has the GPU to itself
    and its duration (HIP events, in-kernel span and a kernel trace alike) is its own.  c3 (one
    stream, bound by its longest 20 MB chains: ~175 ms per stream whatever else runs) runs
    twenty steps in flight on twenty contexts with 32 hardware queues and scans capped at 64
    workgroups (12/16/20 streams: 547/590/673 GiB/s, same box; 24 outrun the queues:
    profiles/r5/c3_inflight/); c4/c5 two (the next commit's scan and hashes fill what the chain-bound hash
    leaves: 824 -> 936 / 820 -> 883 GiB/s, profiles/r3/c4_inflight/).  c2's two-in-flight
    throughput is measured after the timed region (``two_in_flight``)."""
    if args.inflight > 0:
        return args.inflight
    if args.path == "put" and args.config == "c3":
        return C3_INFLIGHT
    if args.path == "put" and args.config in ("c4", "c5"):
        return 2
    return 1


def bench_put(args, ctx, c3s):
    np, torch = ctx["np"], ctx["torch"]
    pd, world, rank, local, dev = ctx["pd"], ctx["world"], ctx["rank"], ctx["local"], ctx["dev"]
    params, cdev, rehearse = ctx["params"], ctx["cdev"], ctx["rehearse"]
    from pfs_amd import _lib
    from pfs_amd.cdc import Chunker

    H = Harness(ctx)
    if args.shard:
        sr, sn = (int(x) for x in args.shard.split("/"))
        work = workload(args, sn, sr)
        work.info["shard"] = "rank %d of %d, alone on one GPU" % (sr, sn)
    else:
        work = workload(args, world, rank)
    total = work.total

    S = inflight_for(args)
    batches = []
    for k in range(S):
        try:
            t = torch.empty(total, dtype=torch.uint8, device=dev)
        except torch.OutOfMemoryError:
            if k == 0 or args.inflight > 0:
                raise
            break
        batches.append(t)
    if args.inflight == 0 and len(batches) > 1:
        # keep headroom for the contexts' own device buffers (segments, entries, refs)
        free, _ = torch.cuda.mem_get_info(dev)
        if free < (4 << 30):
            batches.pop()
            torch.cuda.empty_cache()
    S = len(batches)
    steps, warmup, steps_note = plan_steps(args.steps, args.warmup, S)
    # host ahead: the GPU still runs one step at a time (each step's stream waits for all of
    # the previous step's work), but the next step is already enqueued on a second context
    # over the same input when the current one completes, so the host-side wait, result
    # copy and launch of a step no longer sit between two steps on the GPU
    ahead = S == 1 and (args.host_ahead == 1 or (args.host_ahead < 0 and args.config == "c2"
                                                 and args.path == "put"))
    NC = 2 if ahead else S
    chunkers = [Chunker(params, device=local, ref_ids=args.ref_ids) for _ in range(NC)]
    if S > 1 and args.hash_order == "serial":  # each hash after the previous step's hash
        for k in range(S):
            chunkers[k].order_hash_after(chunkers[(k - 1) % S])
    for k, t in enumerate(batches):
        fill(chunkers[k], t, work)  # every step: the same workload
    if args.path == "get":
        from .get import bench_get
        return bench_get(args, ctx, chunkers[0], batches[0], work)

    chunker, data = chunkers[0], batches[0]
    gather = world > 1 or args.config != "c2"  # the commit's / stream's index on rank 0
    torch.cuda.synchronize()
    steps_t = []   # per timed step: the library's timings dict
    done_at = []   # completion times of the timed steps
    gather_ms = []  # per timed step: the index gather to rank 0 (host wall clock)
    gstats = {}
    pending = [False] * NC
    last = {}

    def finish(k, record):
        """Wait for context k's step; its records and timings (copies: the context can take
        its next step at once)."""
        res = chunkers[k].wait()
        pending[k] = False
        if record:
            steps_t.append(chunkers[k].timings())
            done_at.append(time.perf_counter())
        last[k] = res
        return res

    def gather_step(res, record):
        """The step's chunk-ref index to rank 0.  Called after the next step is enqueued, so
        the GPU has work queued while the host waits on the collective (whose kernels may
        wait for CUs behind that step's scan)."""
        if not gather:
            return
        segs = res.segments.copy()
        segs["file"] = work.gid[segs["file"]].astype(np.uint32)
        if world > 1:
            # counts first, then each rank's live records point to point to rank 0
            g0 = time.perf_counter()
            last["index"] = pd.gather_index_to_root(segs, device=cdev, stats=gstats)
            if record:
                gather_ms.append((time.perf_counter() - g0) * 1e3)
        else:
            last["index"] = segs

    seq = [0]  # the context rotation continues across the warmup and timed runs: restarting
    # it at context 0 after an odd warmup left the two steps serialised on the GPU

    def run(nsteps, record):
        for _ in range(nsteps):
            k = seq[0] % NC
            seq[0] += 1
            done = finish(k, record) if pending[k] else None
            if ahead:  # after everything the other context has enqueued (the previous step)
                chunkers[k].wait_for(chunkers[(k + 1) % NC])
            chunkers[k].scan_async(batches[k % S], work.offs)
            pending[k] = True
            if done is not None:
                gather_step(done, record)
        for j in range(NC):  # drain in launch order
            kk = (seq[0] + j) % NC
            if pending[kk]:
                gather_step(finish(kk, record), record)

    run(warmup, False)
    elapsed = H.timed(lambda k: run(k, True), steps)
    res = last[0]
    bytes_step = H.sum_over_ranks(total)

    intervals = [(b - a) * 1e3 for a, b in zip([H.t0] + done_at[:-1], done_at)]
    kmed = {name: med([s[name] for s in steps_t]) for name in steps_t[0]} if steps_t else {}
    kmean = {name: round(sum(s[name] for s in steps_t) / len(steps_t), 4)
             for name in steps_t[0]} if steps_t else {}
    tj = load_traffic(args, work)

    def roof(ms, kernel, traffic_key=None, nbytes=None):
        nbytes = total if nbytes is None else nbytes
        ach = nbytes / (ms * 1e-3) / 1e9 if ms and ms > 0 else 0.0
        r = {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
             "bytes_per_launch": nbytes, "avg_launch_ms": round(ms, 4) if ms else None,
             "kernel": kernel}
        if tj and traffic_key and tj.get(traffic_key):
            r["traffic"] = tj[traffic_key]
            r["traffic_source"] = tj["_source"] + " (FETCH_SIZE x 2, per launch)"
        return r

    # the dominant kernel's duration: HIP events around its launch on the library's stream,
    # mean over the timed launches (= a kernel trace's per-launch duration when one step is
    # in flight); the in-kernel span (first wavefront start to last wavefront end) beside it
    hash_ms = kmean.get("hash")
    scan_ms = kmean.get("scan")
    dom_hash = (hash_ms or 0) >= (scan_ms or 0)
    roofline = roof(hash_ms, "blake2b_kernel", "blake2b_kernel") if dom_hash else \
        roof(scan_ms, "cdc_scan_kernel", "cdc_scan_kernel")
    roofline["duration_source"] = ("HIP events around the launch on the library's stream, mean "
                                   "over the %d timed launches, %d step(s) in flight%s"
                                   % (len(steps_t), S, " (the host one step ahead)" if ahead
                                      else ""))
    roofline["span_ms"] = kmean.get("hash_span" if dom_hash else "scan_span")
    if args.ref_ids and kmean.get("ref_ids", 0) > (hash_ms or 0):
        roofline = roof(kmean["ref_ids"], "blake2b_kernel<kModeRefId> (ChaCha20 + BLAKE2b of "
                                          "the ciphertext; HIP events)")
    # the scan rolls only the bytes that can hold a cut (the first min - 1 bytes of a file
    # never do: writer.go:167-170), so its per-launch bytes are the rolled ones
    rolled = chunkers[0].last_scan_bytes()
    smode = chunkers[0].last_scan_mode()
    roofline_cdc = roof(scan_ms, "cdc_scan_kernel (its last workgroup compacts the candidates)",
                        "cdc_scan_kernel", nbytes=rolled)
    roofline_cdc["file_bytes_per_launch"] = total
    roofline_cdc["rolled_fraction"] = round(rolled / total, 5) if total else None
    rvalu = {}
    if tj:
        for kern, ms, mhz in (("blake2b_kernel", hash_ms, kmean.get("hash_mhz")),
                              ("cdc_scan_kernel", scan_ms, kmean.get("scan_mhz"))):
            n = tj.get(kern + "_valu")
            if n and ms:
                ach = n / (ms * 1e-3) / 1e9
                rvalu[kern] = {"bound": "valu-issue", "achieved": round(ach, 1),
                               "peak": VALU_PEAK_GIPS, "unit": "G wave-instr/s",
                               "frac": round(ach / VALU_PEAK_GIPS, 4), "valu_per_launch": n,
                               "source": tj["_source"]}
                if mhz:  # the same ceiling at the clock the kernel actually ran at (DVFS)
                    pk = SIMDS * mhz * 1e-3 / 4.0
                    rvalu[kern].update({"clock_mhz": round(mhz, 1),
                                        "peak_at_clock": round(pk, 1),
                                        "frac_at_clock": round(ach / pk, 4)})

    info = dict(work.info)
    if c3s:
        info["scan_grid"] = _lib.get_knob("PFSCDC_SCAN_GRID")
    info.update({"steps_in_flight": S, "host_ahead": ahead,
                 "params": {"average_bits": params.average_bits, "seed": params.seed,
                            "min": params.min_chunk, "max": params.max_chunk},
                 "gpu_max_hw_queues": ctx["hwq"],
                 # the scan's skipping as the library did it in the last step
                 # (pfscdc_last_scan_mode): the first min - 1 bytes of each file, and past every
                 # settled cut
                 "scan_skip": {"first_min": bool(smode & _lib.SCAN_SKIPPED_FIRST_MIN),
                               "past_settled_cuts": bool(smode & _lib.SCAN_SKIPPED_CUTS)},
                 "parallelism": ("%s-sharded x%d, chunk-ref index gathered to rank 0 every "
                                 "step (%s: counts all-gathered, live records sent point to "
                                 "point)" % ("file" if args.config == "c2" else "fileset",
                                             world, "gloo" if rehearse else "RCCL"))
                 if world > 1 else "single GPU"})
    out = H.line(METRIC, bytes_step, steps, warmup, elapsed, work.scaling, info,
                 ref_ids=bool(args.ref_ids), segments_per_step=int(len(res.segments)),
                 ms_per_step_median=med(intervals), kernel_ms=kmean, kernel_ms_median=kmed,
                 note="kernel_ms: per step on this rank; scan/select/hash = HIP events on the "
                      "library's stream (with steps in flight they include waiting for CUs "
                      "behind the other step), scan_span/hash_span = the kernels' own execution "
                      "spans (first wavefront start to last wavefront end); the hash is "
                      "VALU-issue bound, not HBM bound (DESIGN.md §4)",
                 cdc_only_gib_s=round(total / (scan_ms * 1e-3) / GIB, 2) if scan_ms else None,
                 hash_only_gib_s=round(total / (hash_ms * 1e-3) / GIB, 2) if hash_ms else None,
                 roofline=roofline, roofline_cdc=roofline_cdc)
    if steps_note:
        out["steps_requested"], out["warmup_requested"] = args.steps, args.warmup
        out["steps_rule"] = steps_note
    if rvalu:
        out["roofline_valu"] = rvalu
    if S > 1:
        # the rate once the pipeline is full (the whole-region value above includes the fill
        # and the drain: with every stream started at t0 they end together, a burst)
        out["steady_state"] = steady_state(H.t0, done_at, S, total * world)
        # after the timed region: steps alone on the GPU (median of 3), so the kernels' own
        # durations can be read beside the overlapped ones above
        iso, walls = [], []
        for _ in range(3):
            w0 = time.perf_counter()
            chunkers[0].scan_async(batches[0], work.offs)
            chunkers[0].wait()
            walls.append((time.perf_counter() - w0) * 1e3)
            iso.append(chunkers[0].timings())
        im = {name: med([s[name] for s in iso]) for name in iso[0]}
        out["kernel_ms_isolated"] = im
        # one step alone, host to host: the per-stream latency the steps in flight hide
        out["one_step_alone"] = {"value": round(total / (med(walls) * 1e-3) / GIB, 3),
                                 "unit": "GiB/s", "ms": med(walls),
                                 "note": "one step with nothing else in flight (median of 3)"}
        ri = roof(im["hash_span"], "blake2b_kernel")
        rc = roof(im["scan_span"], "cdc_scan_kernel")
        out["roofline_isolated"] = {"hash": ri, "scan": rc,
                                    "note": "median of 3 steps with nothing else in flight, "
                                            "after the timed region"}

    if args.config in ("c4", "c5") and work.group > 1:
        # the literal configuration beside the grouped one: ONE commit per step over the N GPUs
        # (copy 0 of this rank's share: strong scaling, bound by its longest chains)
        out["single_commit"] = single_commit(args, work, chunkers[0], batches[0], H)
    if rank == 0 and not gather:  # c2 at N = 1: the step's own index
        idx = res.segments.copy()
        idx["file"] = work.gid[idx["file"]].astype(np.uint32)
        last["index"] = idx
    if rank == 0 and "index" in last:
        idx = last["index"]
        if args.config in ("c4", "c5"):  # the commit itself: copy 0 of every rank
            idx = idx[idx["file"] < work.layout.npieces]
        if args.config == "c5":
            out["dedup"] = hit_rate(idx)
        # the gathered chunk-ref index of the commit / stream: equal at every N (c2: N ranks
        # at G batches each = one GPU at N G batches)
        out["index_digest"] = hashlib.blake2b(idx.tobytes(), digest_size=16).hexdigest()
        out["index_segments"] = int(len(idx))
        if world > 1:
            live = int(gstats.get("records", 0)) * idx.dtype.itemsize
            out["index_gather"] = {
                "how": "all-gather of the 8-byte counts, then each rank's live records sent "
                       "point to point to rank 0 (no padding, no other receiver)",
                "backend": "gloo" if rehearse else "nccl (RCCL)",
                "records_per_step": int(gstats.get("records", 0)),
                "live_record_bytes_per_step": live,
                "bytes_received_by_rank0_per_step": int(gstats.get("bytes_received", 0)),
                "count_bytes_per_rank": 8 * world,
                "moved_over_live": round((gstats.get("bytes_received", 0) + 8 * world * world)
                                         / max(live, 1), 4),
                "ms_median": med(gather_ms)}

    # the timed steps are done: release the other steps' inputs and contexts (the e2e
    # contexts below allocate their own device copies)
    for k in range(len(chunkers)):
        if S > 1:
            chunkers[k].order_hash_after(None)
    for k in range(1, len(chunkers)):
        chunkers[k].close()
    del batches[1:]
    torch.cuda.empty_cache()

    solo = rank == 0 and world == 1 and not args.shard
    if solo and not args.no_chain_floor:
        out["chain_floor"] = chain_floor(res, hash_ms, data, params, local, Chunker)
    if solo and args.config == "c2" and S == 1 and not args.no_pipelined:
        out["two_in_flight"] = two_in_flight(work, chunker, data, params, local, Chunker, torch)
    if solo and args.config == "c2" and not args.no_literal:
        out["configs1_literal"] = literal_batch(args, work, chunker, data, params, local,
                                                Chunker, torch)
    if solo and args.config == "c2" and not args.no_e2e:
        out["e2e"] = e2e(args, work, data, params, local, Chunker, torch)
    if solo and not args.no_cpu_baseline:
        par.cpu_baseline(args, work, data, res, params, out, last)
    elif rank == 0 and args.config in ("c2", "c4", "c5") and "index" in last and not args.shard:
        # every N: the first and last piece of every rank regenerated here and run through
        # the oracle, vs the gathered index (no bytes move between ranks)
        out["parity"] = par.sample_parity(args, world, last["index"], work.seed, work.mode,
                                          params)
    H.emit(out)
    H.close()
    chunker.close()


def single_commit(args, work, chunker, data, H):
    """One commit per step (G = 1) on the same ranks and contexts: the step time of the
    configured 100 GiB commit itself over N GPUs (strong scaling), max over ranks."""
    offs0 = work.offs[:work.per_copy + 1]
    total0 = int(offs0[-1])
    part = data[:total0]
    for _ in range(max(1, args.warmup)):
        chunker.scan_async(part, offs0)
        chunker.wait()
    k = max(2, min(args.steps, 4))
    hs = []

    def run(n):
        for _ in range(n):
            chunker.scan_async(part, offs0)
            chunker.wait()
            hs.append(chunker.timings()["hash_span"])

    el = H.timed(run, k)
    nb = H.sum_over_ranks(float(total0))
    return {"value": round(nb * k / el / GIB, 3), "unit": "GiB/s", "ms_per_step": round(el * 1e3 / k, 3),
            "steps": k, "commits_per_step": 1, "scaling": "strong",
            "hash_span_ms_median": med(hs),
            "note": "the same ranks with one commit per step instead of %d: bound by the serial "
                    "BLAKE2b chains of the commit's ~10.7 MB files on each GPU" % work.group}


def chain_floor(res, hash_ms, data, params, local, Chunker):
    """The BLAKE2b per-segment latency bound: a segment is one serial chain, so
    no hash launch can end before its longest segment, hashed alone at one quad's rate.  The
    rate is measured here on one 8 MiB range of the step's input, alone on the GPU."""
    longest = int(res.segments["size"].max()) if len(res.segments) else 0
    n = min(8 << 20, int(data.numel()))
    c = Chunker(params, device=local)
    c.hash_ranges(data, [0], [n])  # warm
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        c.hash_ranges(data, [0], [n])
        ts.append(time.perf_counter() - t0)
    c.close()
    rate = n / min(ts)
    floor_ms = longest / rate * 1e3
    return {"longest_segment_bytes": longest, "one_chain_MB_per_s": round(rate / 1e6, 1),
            "floor_ms": round(floor_ms, 2),
            "hash_ms": round(hash_ms, 3) if hash_ms else None,
            "hash_over_floor": round(hash_ms / floor_ms, 3) if hash_ms and floor_ms else None,
            "note": "floor = longest segment / one chain's rate (one quad alone, 8 MiB range of "
                    "this input, best of 3 incl. launch); the hash launch cannot end earlier"}


def _alternate(ctxs, bufs, offs, n):
    """n steps alternating over len(ctxs) contexts (one step in flight per context); seconds."""
    busy = [False] * len(ctxs)
    t0 = time.perf_counter()
    for i in range(n):
        k = i % len(ctxs)
        if busy[k]:
            ctxs[k].wait()
        ctxs[k].scan_async(bufs[k], offs)
        busy[k] = True
    for j in range(len(ctxs)):
        k = (n + j) % len(ctxs)
        if busy[k]:
            ctxs[k].wait()
    return time.perf_counter() - t0


def two_in_flight(work, chunker, data, params, local, Chunker, torch):
    """After the timed region: the same steps with two in flight (a second context on its own
    stream over its own copy of the input), so the next step's scan fills the CUs this step's
    hash frees as its queue drains.  Reported beside the contract's one-at-a-time value."""
    try:
        data2 = torch.empty_like(data)
    except torch.OutOfMemoryError:
        return {"skipped": "HBM cannot hold a second input"}
    data2.copy_(data)
    other = Chunker(params, device=local)
    pair, bufs = [chunker, other], [data, data2]
    n = 10
    _alternate(pair, bufs, work.offs, 2)  # warm
    torch.cuda.synchronize()
    el = _alternate(pair, bufs, work.offs, n)
    other.close()
    del data2
    torch.cuda.empty_cache()
    return {"value": round(work.total * n / el / GIB, 3), "unit": "GiB/s",
            "ms_per_step": round(el * 1e3 / n, 3), "steps": n,
            "note": "two steps in flight on two contexts (hash kernels free to share CUs); "
                    "per-kernel durations are then not a kernel's own, so the contract line "
                    "runs one step at a time"}


def literal_batch(args, work, chunker, data, params, local, Chunker, torch):
    """BASELINE configs[1] exactly as worded: ONE batch of 1024 x 4 MiB per step, no
    aggregation (chain-latency bound: ~1,366 serial BLAKE2b chains fill 1/12 of the GPU)."""
    n = args.files
    sb = int(work.offs[n])
    offs = work.offs[:n + 1]
    view = data[:sb]
    chunker.scan(view, offs)
    torch.cuda.synchronize()
    reps = 6
    t0 = time.perf_counter()
    hs = []
    for _ in range(reps):
        chunker.scan(view, offs)
        hs.append(chunker.timings()["hash_span"])
    serial = (time.perf_counter() - t0) / reps
    # two contexts on two streams alternating (one batch each in flight)
    other = Chunker(params, device=local)
    other.scan(view, offs)
    torch.cuda.synchronize()
    piped = _alternate([chunker, other], [view, view], offs, reps * 2) / (reps * 2)
    other.close()
    # many batches in flight: LITERAL_INFLIGHT contexts (one stream and hardware queue each),
    # every call still one configs[1] batch; the batches' ~4 MiB chains overlap instead of
    # aggregating into one launch.  Steady state: 4 rounds of the contexts after one round.
    from pfs_amd import _lib
    k = args.literal_inflight if args.literal_inflight > 0 else LITERAL_INFLIGHT
    # scans capped at C3_SCAN_GRID workgroups, as for c3's streams: a full-width scan would
    # wait for CUs the other batches' chain-bound hashes hold (12 batches uncapped 800-873
    # GiB/s, 20 capped 993-1,007, 24 outrun the queues: profiles/r5/literal_inflight/)
    grid0 = _lib.get_knob("PFSCDC_SCAN_GRID")
    _lib.set_knob("PFSCDC_SCAN_GRID", args.literal_scan_grid if args.literal_scan_grid >= 0
                  else C3_SCAN_GRID)
    many = [chunker] + [Chunker(params, device=local) for _ in range(k - 1)]
    _alternate(many, [view] * k, offs, k)
    torch.cuda.synchronize()
    nmany = 4 * k
    piped_k = _alternate(many, [view] * k, offs, nmany) / nmany
    grid_k = _lib.get_knob("PFSCDC_SCAN_GRID")
    _lib.set_knob("PFSCDC_SCAN_GRID", grid0)
    for c in many[1:]:
        c.close()
    return {"value": round(sb / serial / GIB, 3), "unit": "GiB/s",
            "ms_per_batch": round(serial * 1e3, 3),
            "hash_span_ms_median": round(statistics.median(hs), 3),
            "two_in_flight_value": round(sb / piped / GIB, 3),
            "many_in_flight": {"batches_in_flight": k, "scan_grid": grid_k,
                               "value": round(sb / piped_k / GIB, 3),
                               "ms_per_batch": round(piped_k * 1e3, 3),
                               "note": "%d contexts on %d streams, one configs[1] batch per "
                                       "call, %d batches" % (k, k, nmany)},
            "note": "one configs[1] batch (1024 x 4 MiB) per step, device-resident, no "
                    "aggregation: bound by the ~4 MiB serial BLAKE2b chains (DESIGN.md §4)"}


def e2e(args, work, data, params, local, Chunker, torch):
    """one configs[1] batch (4 GiB) per call from pinned host memory"""
    n = args.files
    sbytes = int(work.offs[n])
    host = torch.empty(sbytes, dtype=torch.uint8, pin_memory=True)
    host.copy_(data[:sbytes])
    hnp = host.numpy()
    boffs = work.offs[:n + 1]
    e2e_chunker = Chunker(params, device=local)
    e2e_chunker.scan(hnp, boffs)
    torch.cuda.synchronize()
    n_e2e = 2
    t0 = time.perf_counter()
    for _ in range(n_e2e):
        e2e_chunker.scan(hnp, boffs)
    te = (time.perf_counter() - t0) / n_e2e
    # pipelined: two contexts (two streams) alternate, so batch k+1's H2D copy runs while
    # batch k hashes
    pipe = [e2e_chunker, Chunker(params, device=local)]
    pipe[1].scan(hnp, boffs)
    torch.cuda.synchronize()
    n_pipe = 8
    tp = _alternate(pipe, [hnp, hnp], boffs, n_pipe) / n_pipe
    for c in pipe:
        c.close()
    del host
    return {"value": round(sbytes / tp / GIB, 3), "unit": "GiB/s",
            "ms_per_batch": round(tp * 1e3, 3),
            "serial_value": round(sbytes / te / GIB, 3),
            "note": "configs[1] batches from pinned host memory (hipMemcpyAsync H2D + kernels "
                    "+ records D2H), two contexts on two streams alternating so each batch's "
                    "copy overlaps the previous batch's kernels; serial_value: one batch at a "
                    "time"}
