#!/usr/bin/env python3
"""Benchmark of the MI355X PFS chunk-ingest path (BASELINE.json metric).

Metric: GiB/s of file bytes through CDC rolling hash + per-segment BLAKE2b-256 content hash
with inputs already resident in HBM.  A "step" = one pass of the whole path over the step's
files: candidate scan -> compaction -> cut selection -> LPT order -> BLAKE2b of every
segment -> segment records back on the host (and, for N>1 or --config c5, the gather of the
chunk-ref index: RCCL all-gather for N>1).

Workloads (--config, BASELINE.json configs[i]; all synthetic, generated in HBM):
  c2 (default, the headline): configs[1], batches of 1024 independent 4 MiB buffers.  One
     step = --group such batches (default 32 = 128 GiB resident), because BLAKE2b chains are
     serial and the hash needs ~16K+ segments in flight to fill the GPU.
     N>1: every rank its own 32-batch shard (weak scaling).
  c3: configs[2], one 10 GiB stream per GPU (block-parallel scan with halos; the serial cut
     set is checked against the CPU oracle on the whole stream).
  c4: configs[3], a 100 GiB commit of 10,000 files (10,737,418 B each, +2,400 on the last),
     sharded by file across ranks (strong scaling), RCCL all-gather of the chunk-ref index.
  c5: configs[4], the c4 layout with dedup-heavy bytes: 1 MiB blocks, half of them copies of
     64 pooled blocks (--dedup blocks) or half of the files copies of 64 pooled files
     (--dedup files); reports the segment / byte dedup hit rate of the gathered index.

Extra objects on the JSON line: ``roofline`` (dominant kernel, HIP events on the library's
stream), ``roofline_cdc`` (the scan kernel), ``cpu_baseline`` (C restatement of the
reference chunker on the host cores, rank 0 at N=1), ``e2e`` (pinned host input incl. PCIe
H2D, c2 only), ``parity`` (GPU records == CPU oracle records on a sample of the workload).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU issue ceiling: 1024 SIMDs x 2.4 GHz / 4 cycles per wave64 integer VOP3 instruction
# (profiles/r1_ubench_issue_rates.txt: 4.1-4.3 cycles with 2-4 waves per SIMD)
VALU_PEAK_GIPS = 1024 * 2.4 / 4.0
GIB = float(1 << 30)
C4_FILES, C4_FILE_BYTES, C4_TAIL = 10_000, 10_737_418, 2_400
C3_BYTES = 10 * (1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--files", type=int, default=1024, help="c2: files per configs[1] batch")
    ap.add_argument("--file-bytes", type=int, default=4 << 20, help="c2: bytes per file")
    ap.add_argument("--group", type=int, default=32,
                    help="c2: configs[1] batches per step (one launch group, resident in HBM "
                         "together)")
    ap.add_argument("--dedup", default="blocks", choices=["blocks", "files"], help="c5 layout")
    ap.add_argument("--ref-ids", action="store_true",
                    help="also compute every chunk's Ref (Id = BLAKE2b(ChaCha20_dek(chunk)), "
                         "§8 next row 1) inside the step")
    ap.add_argument("--path", default="put", choices=["put", "get", "commit", "uw", "rechunk"],
                    help="put: the ingest path (default); get: chunk.Get of the step's chunks "
                         "(verify BLAKE2b of the stored bytes against Ref.Id, ChaCha20 "
                         "decrypt), §8 next row 3, device-resident in and out; commit: the "
                         "pachd data plane, §8 next rows 1-3: files cut into filesets at "
                         "--mem-threshold bytes, one chunk.Writer stream per fileset (Annotate "
                         "cut, CDC cuts, Close), chunk.Create (Ref.Id/Dek) per formed chunk")
    ap.add_argument("--uw-bytes", type=int, default=8 << 30,
                    help="uw: host bytes Put through the UnorderedWriter per step")
    ap.add_argument("--rechunk-writers", type=int, default=10,
                    help="rechunk: writers the file was written by (TestStableHash shape)")
    ap.add_argument("--mem-threshold", type=int, default=10 ** 9,
                    help="commit: UnorderedWriter memThreshold (storage.go:23, 1e9)")
    ap.add_argument("--seed", type=int, default=-1, help="data seed (default: per config)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="steps in flight (one GPU context + input buffer each; --path commit: "
                         "one context + host thread each over the step's one input buffer); "
                         "0 = auto: 2 for --path put on c2/c3 (1 if HBM cannot hold 2 inputs), else 1")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, affinity)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--traffic-json", default="", help="per-launch HBM bytes from a PMC run")
    return ap.parse_args()


def workload(args, world, rank):
    """This rank's files for one step: (sizes, global id of its first file, seed, synth
    mode, config info, scaling)."""
    from pfs_amd import distributed as pd
    from pfs_amd.cdc import SYNTH_DEDUP_BLOCKS, SYNTH_DEDUP_FILES, SYNTH_RANDOM

    if args.config == "c2":
        G = max(1, args.group)
        n = args.files * G
        seed = 0xC2 if args.seed < 0 else args.seed
        info = {"workload": "configs[1]: batches of %d x %d B independent buffers; %d batches "
                            "per step (one launch group) per GPU" % (args.files, args.file_bytes, G),
                "files_per_step": n, "file_bytes": args.file_bytes, "batches_per_step": G}
        return [args.file_bytes] * n, 0, seed + 1000 * rank, SYNTH_RANDOM, info, "weak"
    if args.config == "c3":
        seed = 0xC3 if args.seed < 0 else args.seed
        info = {"workload": "configs[2]: one %d B stream per GPU" % C3_BYTES,
                "files_per_step": 1, "file_bytes": C3_BYTES}
        return [C3_BYTES], 0, seed + 1000 * rank, SYNTH_RANDOM, info, "weak"
    sizes = [C4_FILE_BYTES] * C4_FILES
    sizes[-1] += C4_TAIL
    b, e = pd.shard_files(sizes, world)[rank]
    mode = SYNTH_RANDOM
    if args.config == "c5":
        mode = SYNTH_DEDUP_BLOCKS if args.dedup == "blocks" else SYNTH_DEDUP_FILES
    seed = (0xC4 if args.config == "c4" else 0xC5) if args.seed < 0 else args.seed
    what = "100 GiB" if args.config == "c4" else "100 GiB dedup-heavy (%s)" % args.dedup
    info = {"workload": "configs[%d]: %s commit of %d files (%d B each, +%d on the last), "
                        "sharded by file over %d GPU(s)"
                        % (3 if args.config == "c4" else 4, what, C4_FILES, C4_FILE_BYTES,
                           C4_TAIL, world),
            "files_per_step": e - b, "files_total": C4_FILES}
    if args.config == "c5":
        info["dedup"] = ("1 MiB blocks, p=1/2 a copy of one of 64 pooled blocks"
                         if args.dedup == "blocks" else
                         "whole files, p=1/2 a copy of one of 64 pooled files")
    return sizes[b:e], b, seed, mode, info, "strong"


def fill(chunker, tensor, sizes, fbase, seed, mode, np):
    """Generate this rank's files; file f of the shard is file fbase + f of the commit (the
    generator keys bytes by file index, so empty files are put in front of the shard)."""
    offs = np.zeros(fbase + len(sizes) + 1, dtype=np.uint64)
    offs[fbase + 1:] = np.cumsum(np.asarray(sizes, dtype=np.uint64))
    chunker.fill_synthetic(tensor, offs, seed, mode)


def local_index(segments, fbase):
    out = segments.copy()
    out["file"] = out["file"] + fbase
    return out


def hit_rate(index):
    """Fraction of segments (and bytes) whose BLAKE2b digest appeared earlier in commit
    order: the chunk-level dedup a content-addressed store gets from these DataRefs."""
    seen = set()
    hit_s = hit_b = 0
    for h, size in zip(index["hash"], index["size"]):
        key = h.tobytes()
        if key in seen:
            hit_s += 1
            hit_b += int(size)
        else:
            seen.add(key)
    nb = int(index["size"].sum()) if len(index) else 0
    return {"segments": int(len(index)), "segment_hit_rate": round(hit_s / max(len(index), 1), 5),
            "byte_hit_rate": round(hit_b / max(nb, 1), 5), "unique_digests": len(seen)}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from pfs_amd.cdc import ChunkParams, Chunker
    from pfs_amd import distributed as pd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # PFS_BENCH_REHEARSE=1: rehearse the N>1 path with every rank on the box's device(s) and
    # gloo (RCCL refuses two ranks on one GPU); the driver's scaling runs use RCCL.
    rehearse = os.environ.get("PFS_BENCH_REHEARSE") == "1"
    if rehearse:
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    cdev = torch.device("cpu") if rehearse else dev  # collectives' tensors

    params = ChunkParams()  # reference defaults: avgBits 23, seed 1, min 1 MB, max 20 MB
    sizes, fbase, seed, mode, info, scaling = workload(args, world, rank)
    nfiles = len(sizes)
    offs = np.zeros(nfiles + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(np.asarray(sizes, dtype=np.uint64))
    total = int(offs[-1])
    # parity / CPU-baseline sample: the first configs[1] batch (c2), the whole stream (c3),
    # or the shard's first ~4 GiB of files (c4/c5)
    if args.config == "c2":
        sfiles = min(args.files, nfiles)
    elif args.config == "c3":
        sfiles = 1
    else:
        sfiles = min(nfiles, max(1, int((4 << 30) // max(sizes[0], 1))))
    sbytes = int(offs[sfiles])

    # Two steps in flight (two contexts on two streams, one resident input each): the next
    # step's scan starts while this step's hash drains its longest chains (c2 +6%, c3 2x).
    # c4/c5 hashes are ~20K chains of up to 10.7 MB that already fill the GPU: two of them
    # side by side only stretch each other (598-645 vs 667-669 GiB/s), so one step there.
    S = args.inflight if args.inflight > 0 else (
        2 if args.path == "put" and args.config in ("c2", "c3") else 1)
    batches = []
    for k in range(S if args.path != "commit" else 1):
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
    if args.path != "commit":
        S = len(batches)
    chunkers = [Chunker(params, device=local, ref_ids=args.ref_ids) for _ in range(S)]
    for k, t in enumerate(batches):
        fill(chunkers[k], t, sizes, fbase, seed, mode, np)  # every step: the same workload
    chunker, data = chunkers[0], batches[0]
    # all_gather_into_tensor needs equal blocks: the capacity of the largest shard
    cap = max(pd.max_segments(workload(args, world, r)[0], params.min_chunk) for r in range(world))
    gather = world > 1 or args.config == "c5"
    torch.cuda.synchronize()
    acc = {"scan": 0.0, "compact": 0.0, "select": 0.0, "hash": 0.0, "total": 0.0}
    if args.ref_ids:
        acc["ref_ids"] = 0.0
    pending = [False] * S
    last = {}

    def finish(k, record):
        res = chunkers[k].wait()
        pending[k] = False
        if gather:
            last["index"] = pd.gather_index(res.segments, fbase, cap, device=cdev) \
                if world > 1 else local_index(res.segments, fbase)
        if record:
            for name, v in chunkers[k].timings().items():
                acc[name] += v
        last[k] = res
        return res

    seq = [0]  # the context rotation continues across the warmup and timed runs: restarting
    # it at context 0 after an odd warmup left the two steps serialised on the GPU

    def run(nsteps, record):
        for i in range(nsteps):
            k = seq[0] % S
            seq[0] += 1
            if pending[k]:
                finish(k, record)
            chunkers[k].scan_async(batches[k], offs)
            pending[k] = True
        for j in range(S):  # drain in launch order
            kk = (seq[0] + j) % S
            if pending[kk]:
                finish(kk, record)

    if args.path == "get":
        return bench_get(args, world, rank, local, dev, chunkers[0], batches[0], offs, total,
                         info, scaling, params, np, torch, dist)
    if args.path == "rechunk":
        return bench_rechunk(args, world, rank, dev, chunkers[0], batches[0], info, scaling,
                             params, np, torch, dist)
    if args.path == "uw":
        return bench_uw(args, world, rank, dev, chunkers[0], batches[0], sizes, info, scaling,
                        params, np, torch, dist)
    if args.path == "commit":
        return bench_commit(args, world, rank, dev, chunkers, batches[0], sizes, total, info,
                            scaling, params, np, torch, dist)

    run(args.warmup, False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, True)
    res = last[0]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    bytes_step = total
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        bt = torch.tensor([total], dtype=torch.float64, device=cdev)
        dist.all_reduce(bt, op=dist.ReduceOp.SUM)
        bytes_step = int(bt.item())

    K = max(args.steps, 1)
    avg = {k: v / K for k, v in acc.items()}
    value = float(bytes_step) * args.steps / elapsed / GIB
    ms_per_step = elapsed * 1e3 / K

    def roof(ms):
        ach = total / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                "bytes_per_launch": total, "avg_launch_ms": round(ms, 4)}

    dom = "hash" if avg["hash"] >= avg["scan"] else "scan"
    roofline = roof(avg[dom])
    roofline["kernel"] = {"hash": "blake2b_kernel", "scan": "cdc_scan_kernel"}[dom]
    if args.ref_ids and avg["ref_ids"] > avg[dom]:
        roofline = roof(avg["ref_ids"])
        roofline["kernel"] = "blake2b_kernel<true> (ChaCha20 + BLAKE2b of the ciphertext)"
    roofline_cdc = roof(avg["scan"])
    roofline_cdc["kernel"] = "cdc_scan_kernel"
    rvalu = {}
    if args.traffic_json and os.path.exists(args.traffic_json):
        tj = json.load(open(args.traffic_json))
        roofline["traffic"] = tj.get(roofline["kernel"])
        roofline_cdc["traffic"] = tj.get("cdc_scan_kernel")
        # the ceiling that binds both kernels: VALU issue (instructions from the PMC pass)
        for kern, ms in (("blake2b_kernel", avg["hash"]), ("cdc_scan_kernel", avg["scan"])):
            n = tj.get(kern + "_valu")
            if n and ms > 0:
                ach = n / (ms * 1e-3) / 1e9
                rvalu[kern] = {"bound": "valu-issue", "achieved": round(ach, 1),
                               "peak": VALU_PEAK_GIPS, "unit": "G wave-instr/s",
                               "frac": round(ach / VALU_PEAK_GIPS, 4), "valu_per_launch": n}

    info.update({"steps_in_flight": S,
                 "params": {"average_bits": params.average_bits, "seed": params.seed,
                            "min": params.min_chunk, "max": params.max_chunk},
                 "parallelism": "file-sharded x%d, RCCL all-gather of chunk-ref index" % world
                 if world > 1 else "single GPU"})
    out = {
        "metric": "GiB/s device-resident CDC rolling-hash + chunk content-hash",
        "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 bytes generated in HBM)",
        "ref_ids": bool(args.ref_ids),
        "config": info,
        "segments_per_step": int(len(res.segments)),
        "kernel_ms": {k: round(v, 4) for k, v in avg.items()},
        "note": "kernel_ms / roofline durations are per step on this rank (HIP events on the "
                "library's stream); the hash is VALU-issue bound, not HBM bound (DESIGN.md §4)",
        "cdc_only_gib_s": round(total / (avg["scan"] * 1e-3) / GIB, 2) if avg["scan"] else None,
        "roofline": roofline,
        "roofline_cdc": roofline_cdc,
    }
    if rvalu:
        out["roofline_valu"] = rvalu
    if S > 1:
        # after the timed region: one step alone on the GPU, so the kernels' own durations
        # (and rooflines) can be read beside the overlapped ones above
        chunkers[0].scan_async(batches[0], offs)
        chunkers[0].wait()
        iso = {k: round(v, 4) for k, v in chunkers[0].timings().items()}
        out["kernel_ms_isolated"] = iso
        ri = roof(iso["hash"])
        ri["kernel"] = "blake2b_kernel"
        rc = roof(iso["scan"])
        rc["kernel"] = "cdc_scan_kernel"
        out["roofline_isolated"] = {"hash": ri, "scan": rc,
                                    "note": "one step with nothing else in flight, after the "
                                            "timed region; not the headline measurement"}

    if gather and rank == 0 and "index" in last:
        out["dedup"] = hit_rate(last["index"])

    # the timed steps are done: release the other steps' inputs and contexts (the e2e
    # contexts below allocate their own device copies)
    for k in range(1, len(chunkers)):
        chunkers[k].close()
    del batches[1:]
    torch.cuda.empty_cache()

    if rank == 0 and world == 1 and args.config == "c2" and not args.no_e2e:
        # one configs[1] batch (4 GiB) per call from pinned host memory
        host = torch.empty(sbytes, dtype=torch.uint8, pin_memory=True)
        host.copy_(data[:sbytes])
        hnp = host.numpy()
        boffs = offs[:sfiles + 1]
        e2e_chunker = Chunker(params, device=local)
        e2e_chunker.scan(hnp, boffs)
        torch.cuda.synchronize()
        n_e2e = 2
        t0 = time.perf_counter()
        for _ in range(n_e2e):
            e2e_chunker.scan(hnp, boffs)
        te = (time.perf_counter() - t0) / n_e2e
        # pipelined: two contexts (two streams) alternate, so batch k+1's H2D copy runs
        # while batch k hashes
        pipe = [e2e_chunker, Chunker(params, device=local)]
        pipe[1].scan(hnp, boffs)
        n_pipe, busy = 8, [False, False]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n_pipe):
            k = i % 2
            if busy[k]:
                pipe[k].wait()
            pipe[k].scan_async(hnp, boffs)
            busy[k] = True
        for k in range(2):
            if busy[(n_pipe + k) % 2]:
                pipe[(n_pipe + k) % 2].wait()
        tp = (time.perf_counter() - t0) / n_pipe
        out["e2e"] = {"value": round(sbytes / tp / GIB, 3), "unit": "GiB/s",
                      "ms_per_batch": round(tp * 1e3, 3),
                      "serial_value": round(sbytes / te / GIB, 3),
                      "note": "configs[1] batches from pinned host memory (hipMemcpyAsync H2D + "
                              "kernels + records D2H), two contexts on two streams alternating "
                              "so each batch's copy overlaps the previous batch's kernels; "
                              "serial_value: one batch at a time"}
        for c in pipe:
            c.close()
        del host

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import chunker as och
        from oracle import coracle

        threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        hdata = data[:sbytes].cpu().numpy()
        p = och.Params(params.average_bits, params.seed, params.min_chunk, params.max_chunk)
        soffs = offs[:sfiles + 1]
        warm = min(sbytes, 1 << 20)
        coracle.segment_files(hdata[:warm], [0, warm], p)  # load + warm
        t0 = time.perf_counter()
        segs, begin = coracle.segment_files(hdata, soffs, p, nthreads=threads)
        tc = time.perf_counter() - t0
        used = min(threads, sfiles)
        ns1 = max(1, min(sfiles, 32))
        if sfiles > 1:
            t0 = time.perf_counter()
            coracle.segment_files(hdata[:int(offs[ns1])], offs[:ns1 + 1], p, nthreads=1)
            t1 = int(offs[ns1]) / (time.perf_counter() - t0) / GIB
        else:
            t1 = sbytes / tc / GIB
        import platform
        cpu_model = platform.processor() or ""
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
        what = {"c2": "the step's first configs[1] batch", "c3": "the whole stream"}.get(
            args.config, "the shard's first files")
        out["cpu_baseline"] = {
            "value": round(sbytes / tc / GIB, 3), "unit": "GiB/s", "cores": used,
            "kind": "port",
            "sample": "%d file(s), %d B (%s) on %d thread(s), files spread over threads; "
                      "single-thread rate from %d file(s)" % (sfiles, sbytes, what, used, ns1),
            "single_thread_gib_s": round(t1, 4),
            "cpu_model": cpu_model}
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
                a = int(offs[sg["file"]]) + int(sg["offset"])
                rid, dek = och.create_ref_id(hdata[a:a + int(sg["size"])].tobytes())
                ok &= bytes(res.refs[i]["id"]) == rid and bytes(res.refs[i]["dek"]) == dek
            out["parity"]["ref_ids_equal_oracle"] = bool(ok)
            out["parity"]["ref_ids_checked"] = int(nchk)
        if args.config == "c5" and "index" in last:
            # the oracle's digests of the sample give the same hit rate as the GPU's
            ref = local_index(segs, fbase)
            out["parity"]["sample_hit_rate_gpu"] = hit_rate(last["index"][:len(ref)])
            out["parity"]["sample_hit_rate_oracle"] = hit_rate(ref)

    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    chunker.close()


def bench_get(args, world, rank, local, dev, chunker, data, offs, total, info, scaling, params,
              np, torch, dist):
    """Read path: the step's segments are stored chunks (chunk.Create form); one step =
    pfscdc_get_chunks over all of them (verify + decrypt, device in/out)."""
    chunker.set_ref_ids(True)
    res = chunker.scan(data, offs)  # segments + Ref (id, dek): the chunks as stored
    segs = res.segments
    cofs = np.zeros(len(segs) + 1, dtype=np.uint64)
    cofs[1:] = np.cumsum(segs["size"])  # segments tile the batch in (file, offset) order
    assert int(cofs[-1]) == total
    ctext = torch.empty_like(data)
    _, ok0 = chunker.get_chunks(data, cofs, res.refs, out=ctext)  # XOR is its own inverse
    assert not ok0.any() or len(segs) == 0  # plaintext never verifies as the stored form
    out = torch.empty_like(data)
    for _ in range(args.warmup):
        chunker.get_chunks(ctext, cofs, res.refs, out=out)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kms = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, ok = chunker.get_chunks(ctext, cofs, res.refs, out=out)
        kms += chunker.last_get_ms()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    same = bool(ok.all()) and bool(torch.equal(out, data))
    bytes_step = total
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        bt = torch.tensor([total], dtype=torch.float64, device=dev)
        dist.all_reduce(bt, op=dist.ReduceOp.SUM)
        bytes_step = int(bt.item())
    K = max(args.steps, 1)
    ms = kms / K
    ach = total / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    info.update({"path": "get (chunk.Get: verify Ref.Id, ChaCha20 decrypt)",
                 "chunks_per_step": int(len(segs))})
    out_line = {
        "metric": "GiB/s device-resident chunk.Get (verify + decrypt) of stored chunks",
        "value": round(float(bytes_step) * args.steps / elapsed / GIB, 3), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / K, 3), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic plaintext encrypted on the GPU with its own Ref.Dek", "config": info,
        "kernel_ms": {"get": round(ms, 4)},
        "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                     "bytes_per_launch": total, "avg_launch_ms": round(ms, 4),
                     "kernel": "blake2b_kernel<kModeGet>"},
        "parity": {"all_chunks_verified": bool(ok.all()), "plaintext_equals_original": same},
    }
    if rank == 0:
        print(json.dumps(out_line))
    if world > 1:
        dist.destroy_process_group()
    chunker.close()


def commit_layout(sizes, mem_threshold):
    """UnorderedWriter.Put of the files in path order (unordered_writer.go:45-72): the files
    cut into pieces at every mem_threshold bytes, each run of pieces one serialized fileset.
    A Put that fills the threshold exactly re-Adds its path empty in the next fileset.
    Returns (piece sizes, stream_file_begin over pieces)."""
    pieces, streams = [], [0]
    avail = mem_threshold
    for n in sizes:
        n, pos = int(n), 0
        pieces.append(0)  # buffer.Add(p, tag)
        while True:  # io.CopyN(w, r, memAvailable)
            got = min(avail, n - pos)
            pieces[-1] += got
            pos += got
            eof = got < avail
            avail -= got
            if eof:
                break
            if avail == 0:  # serialize, then re-Add the same path
                streams.append(len(pieces))
                avail = mem_threshold
                pieces.append(0)
    if streams[-1] != len(pieces):  # Close serializes the rest
        streams.append(len(pieces))
    return pieces, streams


def bench_commit(args, world, rank, dev, chunkers, data, sizes, total, info, scaling, params,
                 np, torch, dist):
    """pachd data plane on the step's files: pieces / filesets (commit_layout), CDC + DataRef
    hashes (one scan of all pieces), chunk formation per fileset stream (pfscdc_form_chunks),
    chunk.Create of every formed chunk (pfscdc_create_refs: content hash of multi-DataRef
    chunks, dek, ChaCha20 + BLAKE2b of the ciphertext).

    With --inflight S > 1, S contexts (S HIP streams) each run every S-th step from their own
    host thread, so one step's chunk.Create tail (the serial BLAKE2b chains of its largest
    chunks: content hash, then Ref.Id) overlaps the next step's scan and hashes.  The steps
    read the same device buffer (the same files committed again; the library only reads it)."""
    import threading

    S = len(chunkers)
    pieces, streams = commit_layout(sizes, args.mem_threshold)
    poffs = np.zeros(len(pieces) + 1, dtype=np.uint64)
    poffs[1:] = np.cumsum(np.asarray(pieces, dtype=np.uint64))
    assert int(poffs[-1]) == total
    keys = ("scan", "hash", "total", "create", "create_content_hash", "create_ref_id",
            "host_form_ms")
    accs = [dict.fromkeys(keys, 0.0) for _ in range(S)]
    lasts = [{} for _ in range(S)]
    for ch in chunkers:
        ch.set_ref_ids(False)

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
        refs, chash = chunker.create_refs(data, coffs, hashes, known)
        if record:
            acc["create"] += chunker.last_create_ms()
            ct = chunker.last_create_timings()
            acc["create_content_hash"] += ct["content_hash"]
            acc["create_ref_id"] += ct["ref_id"]
        lasts[k].update(res=res, coffs=coffs, known=known, refs=refs)

    errors = []

    def worker(k, nsteps, record):
        try:
            for _ in range(nsteps):
                step(k, record)
        except BaseException as e:  # re-raised on the main thread
            errors.append(e)

    def run(nsteps, record):
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
        worker(k, max(args.warmup, 1) if S > 1 else args.warmup, False)
    if errors:
        raise errors[0]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    bytes_step = total
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        bt = torch.tensor([total], dtype=torch.float64, device=dev)
        dist.all_reduce(bt, op=dist.ReduceOp.SUM)
        bytes_step = int(bt.item())
    K = max(args.steps, 1)
    avg = {name: sum(a[name] for a in accs) / K for name in keys}
    last = lasts[0]
    coffs, known = last["coffs"], last["known"]
    nch = len(coffs) - 1
    info.update({"path": "commit (UnorderedWriter filesets -> chunk.Writer streams -> "
                         "chunk.Create)", "mem_threshold": args.mem_threshold,
                 "filesets_per_step": len(streams) - 1, "pieces_per_step": len(pieces),
                 "chunks_per_step": nch, "multi_dataref_chunks": int(nch - int(known.sum())),
                 "steps_in_flight": S})
    ms = avg["create"]
    ach = total / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    out = {
        "metric": "GiB/s device-resident pachd commit data plane (CDC + DataRef hashes + "
                  "chunk formation + chunk.Create Ref.Id)",
        "value": round(float(bytes_step) * args.steps / elapsed / GIB, 3), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / K, 3), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 bytes generated in HBM)", "config": info,
        "kernel_ms": {name: round(v, 4) for name, v in avg.items()},
        "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                     "bytes_per_launch": total, "avg_launch_ms": round(ms, 4),
                     "kernel": "chunk.Create batch (content hash + dek + ChaCha20/BLAKE2b)"},
    }
    if S > 1:
        out["note"] = ("kernel_ms are per step on its own stream; with %d steps in flight they "
                       "overlap, so ms_per_step < their sum" % S)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["parity"] = commit_parity(data, pieces, streams, poffs, last, params, np)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    for ch in chunkers:
        ch.close()


def bench_uw(args, world, rank, dev, chunker, data, sizes, info, scaling, params, np, torch,
             dist):
    """Host-fed pachd write path: the step's first --uw-bytes of files (host memory) Put
    through the UnorderedWriter (pfs_amd.fileset over pfscdc_uw_*): buffering, 1e9-byte
    filesets, GPU chunk writers with Ref ids and ciphertext upload off, index writers."""
    from pfs_amd import fileset as pf

    offs = np.zeros(len(sizes) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(np.asarray(sizes, dtype=np.uint64))
    nf = int(np.searchsorted(offs, min(args.uw_bytes, int(offs[-1])), side="right")) - 1
    nf = max(1, nf)
    nbytes = int(offs[nf])
    host = data[:nbytes].cpu().numpy()
    views = [memoryview(host[int(offs[f]):int(offs[f + 1])]) for f in range(nf)]
    chunker.close()
    st = pf.Storage(rank % max(1, torch.cuda.device_count()), params, args.mem_threshold)

    split = {"put_ms": 0.0, "close_ms": 0.0}

    def step(record=False):
        w = st.new_unordered_writer()
        t0 = time.perf_counter()
        for f in range(nf):
            w.put("/%016d" % f, "", False, views[f])
        t1 = time.perf_counter()
        prims = w.close()
        if record:
            split["put_ms"] += (t1 - t0) * 1e3
            split["close_ms"] += (time.perf_counter() - t1) * 1e3
        return prims, w

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        prims, w = step(True)
    elapsed = time.perf_counter() - t0
    bytes_step = nbytes
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        bt = torch.tensor([nbytes], dtype=torch.float64, device=dev)
        dist.all_reduce(bt, op=dist.ReduceOp.SUM)
        bytes_step = int(bt.item())
    K = max(args.steps, 1)
    nchunks = sum(1 for fs in w.events for e in fs if e[0] == "chunk" and e[1] == -1)
    info.update({"path": "uw (host-fed UnorderedWriter -> fileset.Writer -> index.Writer)",
                 "files_per_step": nf, "bytes_per_step": nbytes,
                 "mem_threshold": args.mem_threshold, "filesets_per_step": len(prims),
                 "data_chunks_per_step": nchunks})
    out = {
        "metric": "GiB/s host-fed pachd write path (Put -> filesets with chunk Refs and "
                  "multilevel indexes)",
        "value": round(float(bytes_step) * args.steps / elapsed / GIB, 3), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / K, 3), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic bytes in host memory", "config": info,
        "split_ms": {k: round(v / K, 1) for k, v in split.items()},
        "note": "put_ms: the Put loop (one host copy into the fileset arenas, serializations "
                "deferred); close_ms: the grouped GPU write of every fileset plus the indexes",
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def bench_rechunk(args, world, rank, dev, chunker, data, info, scaling, params, np, torch,
                  dist):
    """Re-chunk path (MergeFileReader.Hash, the Writer.Copy machinery): the step's first
    1 GiB as one file written by --rechunk-writers writers (each its own chunk stream,
    ciphertexts uploaded to the in-memory store), then the merged file's hash: Copy of every
    DataRef through a fresh writer, whole aligned chunks passed through, the rest read back
    (chunk.Get on the GPU) and re-rolled.  Checked against the single-writer hash."""
    from pfs_amd import chunk as pc

    nbytes = min(1 << 30, data.numel())
    host = data[:nbytes].cpu().numpy()
    chunker.close()
    store = pc.ChunkStore()
    st = pc.Storage(dev.index or 0, store=store)

    def write(parts):
        refs = []
        w = st.new_writer("w", lambda anns: refs.extend(a.next_data_ref for a in anns
                                                         if a.next_data_ref is not None))
        for part in parts:
            w.annotate(pc.Annotation(data=0))
            w.write(part)
        w.close()
        return refs

    single = write([host])  # the stable-hash reference: one writer
    k = max(1, args.rechunk_writers)
    size = (nbytes + k - 1) // k
    refs = []
    for off in range(0, nbytes, size):
        refs += write([host[off:off + size]])
    want = pc.hash_data_refs([d.hash for d in single], device=dev.index or 0)
    for _ in range(args.warmup):
        pc.merge_file_hash(store, refs, device=dev.index or 0)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        got = pc.merge_file_hash(store, refs, device=dev.index or 0)
    elapsed = time.perf_counter() - t0
    K = max(args.steps, 1)
    edge = sum(1 for d in refs if d.ref.edge)
    info.update({"path": "rechunk (MergeFileReader.Hash of a file written by %d writers)" % k,
                 "file_bytes": nbytes, "data_refs": len(refs), "edge_data_refs": edge,
                 "store_chunks": len(store)})
    out = {
        "metric": "GiB/s of file bytes through MergeFileReader.Hash (Writer.Copy re-chunking)",
        "value": round(nbytes * args.steps / elapsed / GIB, 3), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / K, 3), "higher_is_better": True,
        "scaling": scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 bytes generated in HBM, copied to host)",
        "config": info,
        "parity": {"merged_hash_equals_single_writer_hash": got == want},
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def commit_parity(data, pieces, streams, poffs, last, params, np):
    """The first fileset through the CPU oracle: segments (C restatement), the chunk.Writer
    replay (oracle.chunker), and chunk.Create of a sample of its chunks."""
    from oracle import chunker as och
    from oracle import coracle

    f1 = streams[1]
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
    for i in idx:
        rid, dek = och.create_ref_id(w.chunks[i].data)
        ok &= bytes(last["refs"][i]["id"]) == rid and bytes(last["refs"][i]["dek"]) == dek
    return {"first_fileset_chunk_offsets_equal_oracle": same_cuts, "chunks": n,
            "ref_ids_equal_oracle": bool(ok), "ref_ids_checked": int(len(idx))}


if __name__ == "__main__":
    main()
