#!/usr/bin/env python3
"""Benchmark of the MI355X PFS chunk-ingest path (BASELINE.json metric).

Metric: GiB/s of file bytes through CDC rolling hash + per-segment BLAKE2b-256 content hash
with inputs already resident in HBM.  A "step" = one pass of the whole path over the step's
files: candidate scan (+ compaction) -> cut selection (+ segment compaction, LPT order) ->
BLAKE2b of every segment -> segment records back on the host (and, for N>1 or --config c5,
the gather of the chunk-ref index: an RCCL all-gather for N>1).

Workloads (--config, BASELINE.json configs[i]; all synthetic, generated in HBM):
  c2 (default, the headline): configs[1], batches of 1024 independent 4 MiB buffers.  One
     step = --group such batches (default 32 = 128 GiB resident), because BLAKE2b chains are
     serial and the hash needs ~16K+ segments in flight to fill the GPU.
     N>1: every rank its own 32-batch shard (weak scaling).  The literal one-batch rate is
     reported beside it (``configs1_literal``).
  c3: configs[2], one 10 GiB stream.  N=1: one scan of the stream.  N>1: the stream split in
     equal byte ranges with a 64-byte halo, candidates all-gathered, the serial selection on
     every rank, straddling segments' bytes sent point to point, segments hashed by the rank
     holding their first byte (pfs_amd.distributed.stream_segments; strong scaling).
  c4: configs[3], a 100 GiB commit of 10,000 files (10,737,418 B each, +2,400 on the last),
     cut into serialized filesets of --mem-threshold bytes as pachd's UnorderedWriter does;
     ranks take whole filesets (a file cut at a fileset border is two pieces), so the
     gathered index equals N=1's.  --group G commits per step per rank (auto: enough for
     >= 20K BLAKE2b chains per GPU).
  c5: configs[4], the c4 layout with dedup-heavy bytes: 1 MiB blocks, half of them copies of
     64 pooled blocks (--dedup blocks) or half of the files copies of 64 pooled files
     (--dedup files); reports the segment / byte dedup hit rate of the gathered index.

Extra objects on the JSON line: ``roofline`` (dominant kernel: its execution span measured
inside the kernel, first wavefront start to last wavefront end, = a kernel trace's
duration; traffic and VALU counts from the committed PMC pass of this command when one
exists), ``roofline_cdc`` (the scan kernel), ``cpu_baseline`` (C restatement of the
reference chunker on the host threads the box allots, rank 0 at N=1), ``e2e`` (pinned host
input incl. PCIe H2D, c2 only), ``parity`` (GPU records == CPU oracle records on a sample).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# the legs live in benchkit/ (one module per path, one timing harness); the names the tests
# and tools use stay importable from here
from benchkit.common import (C3_BYTES, C3_INFLIGHT, C3_QUEUES, C3_SCAN_GRID, C4_FILE_BYTES,  # noqa: E402,F401
                             C4_FILES, C4_TAIL, GIB, HBM_PEAK_GBS, LITERAL_INFLIGHT, MIN_CHAINS,
                             Work, auto_group, commit_layout, fill, hit_rate, host_threads,
                             workload)
from benchkit.harness import plan_steps, steady_state  # noqa: E402,F401


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--files", type=int, default=1024, help="c2: files per configs[1] batch")
    ap.add_argument("--file-bytes", type=int, default=4 << 20, help="c2: bytes per file")
    ap.add_argument("--group", type=int, default=0,
                    help="c2: configs[1] batches per step (default 32 = 128 GiB resident); "
                         "c4/c5: commits per step per rank (default: enough for >= 20K "
                         "chains per GPU); c3: 1")
    ap.add_argument("--dedup", default="blocks", choices=["blocks", "files"], help="c5 layout")
    ap.add_argument("--ref-ids", action="store_true",
                    help="also compute every chunk's Ref (Id = BLAKE2b(ChaCha20_dek(chunk)), "
                         "§8 next row 1) inside the step")
    ap.add_argument("--path", default="put",
                    choices=["put", "get", "commit", "uw", "rechunk", "group"],
                    help="put: the ingest path (default); get: chunk.Get of the step's chunks "
                         "(verify BLAKE2b of the stored bytes against Ref.Id, ChaCha20 "
                         "decrypt), §8 next row 3, device-resident in and out; commit: the "
                         "pachd data plane, §8 next rows 1-3: files cut into filesets at "
                         "--mem-threshold bytes, one chunk.Writer stream per fileset (Annotate "
                         "cut, CDC cuts, Close), chunk.Create (Ref.Id/Dek) per formed chunk; "
                         "uw: host-fed UnorderedWriter with indexes; rechunk: Writer.Copy; "
                         "group: one process driving a device group (pfscdc_group_*)")
    ap.add_argument("--members", default="",
                    help="--path group: member devices, e.g. 0,1,2,3 or 0,0,0,0 (default: every "
                         "visible device once); --path uw: the writer's device group (default: "
                         "one GPU)")
    ap.add_argument("--uw-bytes", type=int, default=8 << 30,
                    help="uw: host bytes Put through the UnorderedWriter per step")
    ap.add_argument("--uw-workers", type=int, default=0,
                    help="--path uw: group writers in flight (PFSCDC_UW_WORKERS; default 1)")
    ap.add_argument("--uw-group", type=int, default=0,
                    help="--path uw: bytes of serialized filesets per group write "
                         "(PFSCDC_UW_INFLIGHT; default 32 GiB)")
    ap.add_argument("--rechunk-writers", type=int, default=10,
                    help="rechunk: writers the file was written by (TestStableHash shape)")
    ap.add_argument("--mem-threshold", type=int, default=10 ** 9,
                    help="UnorderedWriter memThreshold (fileset/storage.go:23, 1e9): the "
                         "serialized-fileset size of c4/c5 and of --path commit/uw")
    ap.add_argument("--seed", type=int, default=-1, help="data seed (default: per config)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="steps in flight (one GPU context + input buffer each; --path commit: "
                         "one context + host thread each over the step's one input buffer); "
                         "0 = auto: 4 for --path put on c3, 2 on c4/c5 (fewer if HBM cannot hold "
                         "them), else 1")
    ap.add_argument("--hash-order", default="free", choices=["serial", "free"],
                    help="steps in flight: serial = a step's hash kernel starts after the "
                         "previous step's (scans overlap hash tails; each hash launch has the "
                         "GPU to itself, so its duration is its own); free = hashes of "
                         "different steps may share the CUs")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the host threads the box allots (OMP_NUM_THREADS), else the "
                         "affinity mask")
    ap.add_argument("--cpu-batches", type=int, default=8,
                    help="c2: configs[1] batches in the CPU-baseline sample")
    ap.add_argument("--host-ahead", type=int, default=-1,
                    help="one step at a time on the GPU, the host enqueuing the next step on a "
                         "second context ordered after the current one (1/0; default: on for "
                         "the c2 put path at one step in flight)")
    ap.add_argument("--no-create", action="store_true",
                    help="--path commit: every BLAKE2b of processChunk (DataRef + chunk content "
                         "hashes, one launch) but no chunk.Create (Ref.Id)")
    ap.add_argument("--in-place", type=int, default=-1,
                    help="--path commit: chunk.Create's ciphertext over the plaintext "
                         "(1/0; default: when a ciphertext copy of the step would not fit)")
    ap.add_argument("--commit-hash", default="fused", choices=["fused", "separate"],
                    help="--path commit: DataRef hashes in one launch with the chunks' content "
                         "hashes (pfscdc_commit_refs), or the scan's own hash pass first")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-chain-floor", action="store_true",
                    help="skip the one-chain rate measurement (chain_floor)")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="c2: skip the two-in-flight throughput leg")
    ap.add_argument("--literal-inflight", type=int, default=0,
                    help="configs1_literal: batches in flight in its many-in-flight leg "
                         "(0: the default)")
    ap.add_argument("--literal-scan-grid", type=int, default=-1,
                    help="configs1_literal: PFSCDC_SCAN_GRID for its many-in-flight leg "
                         "(-1: 64, as for c3)")
    ap.add_argument("--no-literal", action="store_true",
                    help="c2: skip the one-batch (unaggregated configs[1]) measurement")
    ap.add_argument("--shard", default="",
                    help="R/N: run rank R's share of an N-GPU job alone on this GPU (no "
                         "collectives): the per-GPU rate an N-GPU run can reach")
    ap.add_argument("--traffic-json", default="",
                    help="per-launch HBM bytes / VALU counts from a PMC run (default: the "
                         "committed profiles/r2 pass of this workload, if any)")
    return ap.parse_args()


def needs_launch(gpus: int, env) -> bool:
    """--gpus N > 1 without a launcher's WORLD_SIZE: this process starts the N ranks itself."""
    return gpus > 1 and "WORLD_SIZE" not in env


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_command(gpus: int, argv, port: int, python: str = sys.executable):
    """torch.distributed.run over this script with the same arguments: one rank per GPU of
    this node, rendezvous on 127.0.0.1."""
    return [python, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
            str(gpus), "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def launch_ranks(gpus: int, argv) -> int:
    """Start the N ranks as a CHILD process (this process has imported nothing that touches
    the GPU and never execs); rank 0's JSON line reaches our stdout through the inherited
    descriptor.  Returns the launcher's exit code."""
    import subprocess
    cmd = launch_command(gpus, argv, free_port())
    print("launching %d ranks: %s" % (gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=dict(os.environ))


def hw_queues_setting(at_least: int = 8) -> int:
    """HIP streams beyond the process's hardware queues (GPU_MAX_HW_QUEUES, HIP's default 4)
    share a queue and run one after the other: c3's streams in flight (one context each) and
    the commit's two chunk sets need a queue per stream.  Raised to
    ``at_least`` (8; 32 for c3's twenty streams) before the first HIP call; a larger setting
    is kept.  The effective value goes into the line's config."""
    try:
        q = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
    except ValueError:
        q = 0
    if q < at_least:
        os.environ["GPU_MAX_HW_QUEUES"] = str(at_least)
        q = at_least
    return q


def c3_streams(args) -> bool:
    """configs[2] on one GPU: several 10 GiB streams in flight, one context each."""
    return args.config == "c3" and args.path == "put" and args.gpus <= 1


def main():
    args = parse()
    if needs_launch(args.gpus, os.environ):
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    c3s = c3_streams(args)
    hwq = hw_queues_setting(C3_QUEUES if c3s or args.config == "c2" else 8)
    if c3s:
        # a step's scan takes one workgroup per CU; with up to twenty chain-bound hash launches
        # of the other streams holding CUs, capped workgroups never wait for them (the
        # PFSCDC_SCAN_GRID knob, read from the environment when the library first uses a knob;
        # an explicit setting is kept)
        os.environ.setdefault("PFSCDC_SCAN_GRID", str(C3_SCAN_GRID))

    import numpy as np
    import torch
    import torch.distributed as dist

    from pfs_amd import distributed as pd
    from pfs_amd.cdc import ChunkParams

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
    cdev = None if rehearse else dev  # collectives' tensors: device (RCCL) or host (gloo)
    ctx = {"np": np, "torch": torch, "dist": dist, "dev": dev, "cdev": cdev, "world": world,
           "rank": rank, "local": local, "pd": pd, "hwq": hwq, "rehearse": rehearse,
           "params": ChunkParams()}  # reference defaults: avgBits 23, seed 1, min 1 MB, max 20 MB
    if args.path == "uw":
        from benchkit.uw import bench_uw
        return bench_uw(args, ctx)
    if args.path == "group":
        from benchkit.group import bench_group
        return bench_group(args, ctx)
    if args.path == "rechunk":
        from benchkit.rechunk import bench_rechunk
        return bench_rechunk(args, ctx)
    if args.path == "commit":
        from benchkit.commit import bench_commit
        return bench_commit(args, ctx)
    if args.config == "c3" and world > 1 and args.path == "put":
        from benchkit.c3split import bench_c3_split
        return bench_c3_split(args, ctx)
    from benchkit.put import bench_put  # put (and get, over the same inputs)
    return bench_put(args, ctx, c3s)


if __name__ == "__main__":
    main()
