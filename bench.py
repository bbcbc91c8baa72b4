#!/usr/bin/env python3
"""Benchmark of the MI355X PFS chunk-ingest path (BASELINE.json metric).

Metric: GiB/s of file bytes through CDC rolling hash + per-segment BLAKE2b-256 content hash
with inputs already resident in HBM.  Workload at N=1 = BASELINE.json configs[1]: 1024
independent 4 MiB buffers (one file = one chunk stream each), synthetic bytes (seeded
splitmix64 stream, see include/pfscdc.h).  A "step" = one pass of the whole path over the
batch: candidate scan -> compaction -> cut selection -> BLAKE2b of every segment -> segment
records back on the host (and, for N>1, the RCCL all-gather of the chunk-ref index).

N>1 (torch.distributed.run, one rank per GPU): every rank owns its own 1024 x 4 MiB shard
of a commit (weak scaling); value = all ranks' bytes / max-over-ranks time.

Extra objects on the JSON line: ``roofline`` (dominant kernel, HIP events on the
library's stream), ``roofline_cdc`` (the scan kernel), ``cpu_baseline`` (C restatement of
the reference chunker on the host cores, rank 0 at N=1), ``e2e`` (pinned host input incl.
PCIe H2D), ``parity`` (GPU records == CPU records on the measured workload).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--files", type=int, default=1024)
    ap.add_argument("--file-bytes", type=int, default=4 << 20)
    ap.add_argument("--seed", type=int, default=0xC2)
    ap.add_argument("--group", type=int, default=32,
                    help="configs[1] batches per step (one launch group, resident in HBM "
                         "together): BLAKE2b chains are serial, so the hash needs ~32K "
                         "segments in flight to fill 1024 SIMDs")
    ap.add_argument("--inflight", type=int, default=1,
                    help="steps in flight (one GPU context + input buffer each)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, affinity)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--traffic-json", default="", help="per-launch HBM bytes from a PMC run")
    return ap.parse_args()


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
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    params = ChunkParams()  # reference defaults: avgBits 23, seed 1, min 1 MB, max 20 MB
    G = max(1, args.group)
    bfiles, fbytes = args.files, args.file_bytes  # one configs[1] batch
    nfiles = bfiles * G                             # files per step
    offs = np.arange(nfiles + 1, dtype=np.uint64) * np.uint64(fbytes)
    total = int(offs[-1])
    bbytes = bfiles * fbytes
    S = max(1, args.inflight)
    chunkers = [Chunker(params, device=local) for _ in range(S)]
    batches = []
    for k in range(S):  # rank r's shard of the commit; batch k = its k-th 1024-file batch
        t = torch.empty(total, dtype=torch.uint8, device=dev)
        chunkers[k].fill_synthetic(t, offs, args.seed + 1000 * rank + k)
        batches.append(t)
    chunker, data = chunkers[0], batches[0]
    cap = pd.max_segments([fbytes] * nfiles, params.min_chunk)
    torch.cuda.synchronize()
    acc = {"scan": 0.0, "compact": 0.0, "select": 0.0, "hash": 0.0, "total": 0.0}
    pending = [False] * S
    last = {}

    def finish(k, record):
        res = chunkers[k].wait()
        pending[k] = False
        if world > 1:
            pd.gather_index(res.segments, rank * nfiles, cap, device=dev)
        if record:
            for name, v in chunkers[k].timings().items():
                acc[name] += v
        last[k] = res
        return res

    def run(nsteps, record):
        for i in range(nsteps):
            k = i % S
            if pending[k]:
                finish(k, record)
            chunkers[k].scan_async(batches[k], offs)
            pending[k] = True
        for k in range(S):  # drain in launch order
            kk = (nsteps + k) % S
            if pending[kk]:
                finish(kk, record)

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
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    K = max(args.steps, 1)
    avg = {k: v / K for k, v in acc.items()}
    bytes_all = float(total) * world * args.steps
    value = bytes_all / elapsed / GIB
    ms_per_step = elapsed * 1e3 / K

    def roof(ms):
        ach = total / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        return {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                "bytes_per_launch": total, "avg_launch_ms": round(ms, 4)}

    dom = "hash" if avg["hash"] >= avg["scan"] else "scan"
    roofline = roof(avg[dom])
    roofline["kernel"] = {"hash": "blake2b_kernel", "scan": "cdc_scan_kernel"}[dom]
    roofline_cdc = roof(avg["scan"])
    roofline_cdc["kernel"] = "cdc_scan_kernel"
    if args.traffic_json and os.path.exists(args.traffic_json):
        tj = json.load(open(args.traffic_json))
        roofline["traffic"] = tj.get(roofline["kernel"])
        roofline_cdc["traffic"] = tj.get("cdc_scan_kernel")

    out = {
        "metric": "GiB/s device-resident CDC rolling-hash + chunk content-hash",
        "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 bytes generated in HBM)",
        "config": {"workload": "configs[1]: batches of %d x %d B independent buffers; %d batches "
                               "per step (one launch group) per GPU" % (bfiles, fbytes, G),
                   "files_per_step": nfiles, "file_bytes": fbytes, "batches_per_step": G,
                   "steps_in_flight": S,
                   "params": {"average_bits": params.average_bits, "seed": params.seed,
                              "min": params.min_chunk, "max": params.max_chunk},
                   "parallelism": "file-sharded x%d, RCCL all-gather of chunk-ref index" % world
                   if world > 1 else "single GPU"},
        "segments_per_step": int(len(res.segments)),
        "kernel_ms": {k: round(v, 4) for k, v in avg.items()},
        "note": "kernel_ms / roofline durations are per step (HIP events on each context's "
                "stream); with steps_in_flight > 1 steps overlap on the GPU",
        "cdc_only_gib_s": round(total / (avg["scan"] * 1e-3) / GIB, 2) if avg["scan"] else None,
        "roofline": roofline,
        "roofline_cdc": roofline_cdc,
    }

    if rank == 0 and world == 1 and not args.no_e2e:
        # PCIe-inclusive: pinned host batch -> H2D -> path -> records back (not `value`)
        # one configs[1] batch (4 GiB) per call, G calls: the host side streams batches
        host = torch.empty(bbytes, dtype=torch.uint8, pin_memory=True)
        host.copy_(data[:bbytes])
        hnp = host.numpy()
        boffs = offs[:bfiles + 1]
        e2e_chunker = Chunker(params, device=local)
        e2e_chunker.scan(hnp, boffs)
        torch.cuda.synchronize()
        n_e2e = 2
        t0 = time.perf_counter()
        for _ in range(n_e2e):
            e2e_chunker.scan(hnp, boffs)
        te = (time.perf_counter() - t0) / n_e2e
        out["e2e"] = {"value": round(bbytes / te / GIB, 3), "unit": "GiB/s",
                      "ms_per_batch": round(te * 1e3, 3),
                      "note": "one configs[1] batch from pinned host memory: hipMemcpyAsync "
                              "H2D + kernels + records D2H, serial (no overlap)"}
        e2e_chunker.close()
        del host

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import chunker as och
        from oracle import coracle

        threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        hdata = data[:bbytes].cpu().numpy()  # the step's first configs[1] batch
        p = och.Params(params.average_bits, params.seed, params.min_chunk, params.max_chunk)
        boffs = offs[:bfiles + 1]
        coracle.segment_files(hdata[:fbytes], offs[:2], p, nthreads=1)  # load/warm
        t0 = time.perf_counter()
        segs, begin = coracle.segment_files(hdata, boffs, p, nthreads=threads)
        tc = time.perf_counter() - t0
        ns1 = max(1, min(bfiles, 32))
        t0 = time.perf_counter()
        coracle.segment_files(hdata[:ns1 * fbytes], offs[:ns1 + 1], p, nthreads=1)
        t1c = time.perf_counter() - t0
        import platform
        cpu_model = platform.processor() or ""
        try:
            for line in open("/proc/cpuinfo"):
                if line.startswith("model name"):
                    cpu_model = line.split(":", 1)[1].strip()
                    break
        except OSError:
            pass
        out["cpu_baseline"] = {
            "value": round(bbytes / tc / GIB, 3), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": "one configs[1] batch (%d x %d B, the step's first) on %d threads; "
                      "single-thread rate from %d files" % (bfiles, fbytes, threads, ns1),
            "single_thread_gib_s": round(ns1 * fbytes / t1c / GIB, 4),
            "cpu_model": cpu_model}
        g = res.segments[:int(res.file_begin[bfiles])]
        same = len(g) == len(segs) and all(np.array_equal(g[f], segs[f]) for f in
                                           ("offset", "size", "file", "flags", "hash"))
        out["parity"] = {"gpu_equals_cpu_oracle": bool(same), "segments": int(len(segs)),
                         "checked": "first configs[1] batch of the last measured step"}

    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    chunker.close()


if __name__ == "__main__":
    main()
