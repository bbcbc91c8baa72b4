"""Checks of a bench line's records against the CPU oracle (test infrastructure: the oracle is
imported only here, after the timed region, as the checker).

- cpu_baseline(): rank 0 at N = 1 times the oracle (the C restatement of the reference
  chunker) on a bounded sample of the step's input and compares the GPU records on it.
- sample_parity(): at any N, rank 0 regenerates on the host the first and last piece of every
  rank (the synthetic bytes are a function of (file, offset, seed), so no bytes move) and
  compares the gathered chunk-ref index entries of those pieces with the oracle's
  (the N > 1 line proves itself).  Reference collection point:
  src/internal/storage/fileset/writer.go:127-149.
- stream_border_parity(): configs[2] split over N ranks; the segments around every rank
  border checked against Writer.roll's cut rule (writer.go:163-189) and BLAKE2b, and the
  segment list tiling the stream.
"""
import os
import time

from .common import GIB, cpu_model, hit_rate, host_threads, workload


def _oracle_params(params):
    from oracle import chunker as och
    return och.Params(params.average_bits, params.seed, params.min_chunk, params.max_chunk)


def sample_pieces(args, world):
    """Rank 0's parity sample at N ranks: the first and last file of every rank's share (c2),
    or the first and last piece of its share of the commit itself (c4/c5: copy 0).
    [(rank, gid, file_id, start, size)]; gid = the piece's id in the gathered index."""
    out = []
    for r in range(world):
        w = workload(args, world, r)
        n = w.per_copy if args.config in ("c4", "c5") else len(w.sizes)
        if n == 0:
            continue
        for i in sorted({0, n - 1}):
            out.append((r, int(w.gid[i]), int(w.ids[i]), int(w.starts[i]), int(w.sizes[i])))
    return out


def compare(got, want):
    """Segment records equal field by field (offset, size, flags, BLAKE2b)."""
    import numpy as np
    if len(got) != len(want):
        return False
    return all(np.array_equal(got[f], want[f]) for f in ("offset", "size", "flags", "hash"))


def sample_parity(args, world, index, seed, mode, params, threads=None):
    """The gathered index entries of sample_pieces() against the oracle (rank 0)."""
    import numpy as np

    from oracle import coracle
    from pfs_amd.cdc import synthetic_piece_bytes

    t0 = time.perf_counter()
    sample = sample_pieces(args, world)
    parts = [synthetic_piece_bytes(f, s, z, seed, mode) for (_, _, f, s, z) in sample]
    offs = np.zeros(len(parts) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts])
    data = np.concatenate(parts) if parts else np.zeros(0, dtype=np.uint8)
    segs, begin = coracle.segment_files(data, offs, _oracle_params(params),
                                        nthreads=threads or host_threads())
    ok, nseg, bad = True, 0, []
    for k, (r, gid, _, _, _) in enumerate(sample):
        want = segs[int(begin[k]):int(begin[k + 1])]
        got = index[index["file"] == np.uint32(gid)]
        got = got[np.argsort(got["offset"], kind="stable")]
        nseg += len(want)
        if not compare(got, want):
            ok = False
            bad.append(gid)
    return {"gpu_equals_cpu_oracle": bool(ok), "segments": int(nseg),
            "pieces": len(sample), "bytes": int(offs[-1]),
            "checked": "first and last piece of each of %d rank(s), regenerated on rank 0 "
                       "and run through the C oracle, vs the gathered index" % world,
            "mismatched_pieces": bad[:8], "seconds": round(time.perf_counter() - t0, 2)}


def rule_check(seg, window, wstart, n, params, cand_fn, hash_fn):
    """One segment [s, e) of a stream against Writer.roll (writer.go:163-189): a cut segment
    ends at the first candidate at or past s + min - 1, else at s + max - 1; an open tail
    (the stream's end) holds no eligible candidate and is shorter than max.  window: the
    stream bytes [wstart, e) with wstart <= s + min - 64 (min >= 64: wstart = s will do)."""
    s, z, flags = int(seg["offset"]), int(seg["size"]), int(seg["flags"])
    e = s + z
    mn, mx = params.min_chunk, params.max_chunk
    if hash_fn(window[s - wstart:e - wstart].tobytes()) != bytes(seg["hash"]):
        return False
    first = None
    if s + mn - 1 < e:
        a = s + mn - 64  # the 64-byte window of position s + min - 1 starts here
        c = cand_fn(window[a - wstart:e - wstart])  # offsets >= 63 of this slice
        if len(c):
            first = a + int(c[0])
    if flags & 2:  # ends on a cut
        return (first == e - 1) or (first is None and z == mx)
    return e == n and first is None and z < mx


def stream_border_parity(segs, n, ranges, seed, params):
    """configs[2] over N ranks: every segment touching a rank border (and its neighbours)
    against the cut rule and BLAKE2b, and the whole list tiling [0, n)."""
    import hashlib

    import numpy as np

    from oracle import coracle
    from pfs_amd.cdc import synthetic_piece_bytes

    t0 = time.perf_counter()
    offs, sizes = segs["offset"].astype(np.int64), segs["size"].astype(np.int64)
    tiles = bool(len(segs)) and int(offs[0]) == 0 and bool(np.all(offs[1:] == offs[:-1] + sizes[:-1])) \
        and int(offs[-1] + sizes[-1]) == n
    p = _oracle_params(params)
    pick = set()
    for (a, _) in ranges[1:]:
        i = int(np.searchsorted(offs, a, side="right")) - 1
        pick.update(j for j in (i - 1, i, i + 1) if 0 <= j < len(segs))
    ok = True
    for j in sorted(pick):
        s, z = int(offs[j]), int(sizes[j])
        # min >= 64: the windows of the eligible positions lie inside the segment's own bytes
        win = synthetic_piece_bytes(0, s, z, seed)
        ok &= rule_check(segs[j], win, s, n, params,
                         lambda b: coracle.candidates(b, p),
                         lambda b: hashlib.blake2b(b, digest_size=32).digest())
    return {"gpu_equals_cpu_oracle": bool(ok and tiles), "segments_tile_stream": tiles,
            "border_segments_checked": len(pick),
            "checked": "the segments around each of %d rank border(s) against Writer.roll's "
                       "cut rule (C oracle candidates) and BLAKE2b; the list tiles the stream"
                       % max(len(ranges) - 1, 0),
            "seconds": round(time.perf_counter() - t0, 2)}


def cpu_baseline(args, work, data, res, params, out, last):
    """The C restatement of the reference chunker (oracle, kind "port") on the host threads
    the box allots, over a bounded sample of the same workload, plus the parity check of the
    GPU records on that sample."""
    import numpy as np

    from oracle import chunker as och
    from oracle import coracle

    threads = args.cpu_threads or host_threads()
    if args.config == "c2":
        sfiles = min(len(work.sizes), args.files * max(1, args.cpu_batches))
        what = "the step's first %d configs[1] batch(es)" % (sfiles // max(args.files, 1))
    elif args.config == "c3":
        sfiles = 1
        what = "the whole stream (one stream: one thread)"
    else:
        sfiles = min(len(work.sizes), max(1, int((16 << 30) // max(work.sizes[0], 1))))
        what = "the first %d pieces of the commit (~16 GiB)" % sfiles
    sbytes = int(work.offs[sfiles])
    hdata = data[:sbytes].cpu().numpy()
    p = _oracle_params(params)
    soffs = work.offs[:sfiles + 1]
    warm = min(sbytes, 1 << 20)
    coracle.segment_files(hdata[:warm], [0, warm], p)  # load + warm
    t0 = time.perf_counter()
    segs, begin = coracle.segment_files(hdata, soffs, p, nthreads=threads)
    tc = time.perf_counter() - t0
    used = min(threads, sfiles)
    ns1 = max(1, min(sfiles, 32))
    if sfiles > 1:
        t0 = time.perf_counter()
        coracle.segment_files(hdata[:int(work.offs[ns1])], work.offs[:ns1 + 1], p, nthreads=1)
        t1 = int(work.offs[ns1]) / (time.perf_counter() - t0) / GIB
    else:
        t1 = sbytes / tc / GIB
    aff = len(os.sched_getaffinity(0))
    out["cpu_baseline"] = {
        "value": round(sbytes / tc / GIB, 3), "unit": "GiB/s", "cores": used,
        "kind": "port",
        "sample": "%d file(s), %d B (%s) on %d thread(s), files spread over threads; "
                  "single-thread rate from %d file(s)" % (sfiles, sbytes, what, used, ns1),
        "single_thread_gib_s": round(t1, 4),
        "host_cpus_visible": aff,
        "threads_note": "threads = the host share the GPU box allots this job "
                        "(OMP_NUM_THREADS); the files are independent, so the rate scales "
                        "per thread up to the socket's cores",
        "cpu_model": cpu_model()}
    g = res.segments[:int(res.file_begin[sfiles])]
    same = len(g) == len(segs) and all(np.array_equal(g[f], segs[f]) for f in
                                       ("offset", "size", "file", "flags", "hash"))
    out["parity"] = {"gpu_equals_cpu_oracle": bool(same), "segments": int(len(segs)),
                     "checked": "the cpu_baseline sample, last measured step"}
    if args.ref_ids:
        nchk = min(16, len(g))
        ok = True
        for i in np.linspace(0, len(g) - 1, nchk).astype(int):
            sg = g[i]
            a = int(work.offs[sg["file"]]) + int(sg["offset"])
            rid, dek = och.create_ref_id(hdata[a:a + int(sg["size"])].tobytes())
            ok &= bytes(res.refs[i]["id"]) == rid and bytes(res.refs[i]["dek"]) == dek
        out["parity"]["ref_ids_equal_oracle"] = bool(ok)
        out["parity"]["ref_ids_checked"] = int(nchk)
    if args.config == "c5" and "index" in last:
        # the oracle's digests of the sample give the same hit rate as the GPU's
        out["parity"]["sample_hit_rate_gpu"] = hit_rate(last["index"][:len(segs)])
        out["parity"]["sample_hit_rate_oracle"] = hit_rate(segs)
