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
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU issue ceiling for the 4-cycle class of wave64 integer ops (VOP3 alignbit/perm/add3,
# 64-bit adds, DPP forms, carry adds: 4.1-4.3 SIMD cycles each at 2 waves per SIMD;
# profiles/r2/valu_issue.txt): 1024 SIMDs x 2.4 GHz / 4.  Plain 32-bit VOP2 ops (xor, add,
# shifts) issue in ~2.1 cycles, so a kernel's own mix sets its exact ceiling.
SIMDS = 1024  # 256 CUs x 4 SIMDs
VALU_PEAK_GIPS = SIMDS * 2.4 / 4.0
GIB = float(1 << 30)
C4_FILES, C4_FILE_BYTES, C4_TAIL = 10_000, 10_737_418, 2_400
C3_BYTES = 10 * (1 << 30)
# BLAKE2b chains per GPU per step for the hash to reach its issue bound (c4 rank 0 of 8 alone
# on one GPU: 16K chains 545 GiB/s, 21K chains 696 GiB/s, N=1's 20.5K 661; profiles/r2/scale/)
MIN_CHAINS = 20480


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
    ap.add_argument("--path", default="put", choices=["put", "get", "commit", "uw", "rechunk"],
                    help="put: the ingest path (default); get: chunk.Get of the step's chunks "
                         "(verify BLAKE2b of the stored bytes against Ref.Id, ChaCha20 "
                         "decrypt), §8 next row 3, device-resident in and out; commit: the "
                         "pachd data plane, §8 next rows 1-3: files cut into filesets at "
                         "--mem-threshold bytes, one chunk.Writer stream per fileset (Annotate "
                         "cut, CDC cuts, Close), chunk.Create (Ref.Id/Dek) per formed chunk; "
                         "uw: host-fed UnorderedWriter with indexes; rechunk: Writer.Copy")
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
    ap.add_argument("--no-literal", action="store_true",
                    help="c2: skip the one-batch (unaggregated configs[1]) measurement")
    ap.add_argument("--shard", default="",
                    help="R/N: run rank R's share of an N-GPU job alone on this GPU (no "
                         "collectives): the per-GPU rate an N-GPU run can reach")
    ap.add_argument("--traffic-json", default="",
                    help="per-launch HBM bytes / VALU counts from a PMC run (default: the "
                         "committed profiles/r2 pass of this workload, if any)")
    return ap.parse_args()


class Work:
    """This rank's input for one step: pieces (files or pieces of files) with their synthetic
    file ids and starts, the global id of its first piece, and the layout info."""

    def __init__(self, sizes, ids, starts, seed, mode, info, scaling, gbase=0, group=1,
                 per_copy=None):
        import numpy as np
        self.sizes = [int(x) for x in sizes]
        self.ids = np.asarray(ids, dtype=np.uint32)
        self.starts = np.asarray(starts, dtype=np.uint64)
        self.seed, self.mode, self.info, self.scaling = seed, mode, info, scaling
        self.gbase, self.group = gbase, group
        self.per_copy = per_copy if per_copy is not None else len(self.sizes)
        self.offs = np.zeros(len(self.sizes) + 1, dtype=np.uint64)
        self.offs[1:] = np.cumsum(np.asarray(self.sizes, dtype=np.uint64))
        # global id of every local piece in the gathered index (copy g of a commit: ids
        # g * pieces_per_commit + piece)
        self.gid = np.arange(len(self.sizes), dtype=np.uint64) + np.uint64(gbase)

    @property
    def total(self) -> int:
        return int(self.offs[-1])


def auto_group(chains_per_copy: int, bytes_per_copy: int, cap: int = 8,
               hbm_budget: int = 180 << 30) -> int:
    """Copies per step so the GPU holds >= MIN_CHAINS BLAKE2b chains, within HBM."""
    g = max(1, math.ceil(MIN_CHAINS / max(chains_per_copy, 1)))
    return max(1, min(g, cap, hbm_budget // max(bytes_per_copy, 1)))


def workload(args, world, rank):
    """This rank's pieces for one step."""
    import numpy as np

    from pfs_amd import distributed as pd
    from pfs_amd.cdc import SYNTH_DEDUP_BLOCKS, SYNTH_DEDUP_FILES, SYNTH_RANDOM

    if args.config == "c2":
        G = args.group if args.group > 0 else 32
        n = args.files * G
        seed = 0xC2 if args.seed < 0 else args.seed
        info = {"workload": "configs[1]: batches of %d x %d B independent buffers; %d batches "
                            "per step (one launch group) per GPU" % (args.files, args.file_bytes, G),
                "files_per_step": n, "file_bytes": args.file_bytes, "batches_per_step": G}
        # rank r holds global files [r n, (r + 1) n) of one synthetic file sequence, so N ranks
        # at G batches each cover the same files as one GPU at N G batches: equal index digests
        return Work([args.file_bytes] * n, np.arange(n) + rank * n, np.zeros(n), seed,
                    SYNTH_RANDOM, info, "weak", gbase=rank * n, group=G, per_copy=args.files)
    if args.config == "c3":
        seed = 0xC3 if args.seed < 0 else args.seed
        a, b = pd.split_stream(C3_BYTES, world)[rank]
        info = {"workload": "configs[2]: one %d B stream%s" % (
                    C3_BYTES, "" if world == 1 else ", split in %d equal byte ranges with a "
                    "64-byte halo (candidates gathered, serial select, border segments sent "
                    "point to point)" % world),
                "files_per_step": 1, "file_bytes": C3_BYTES, "range": [a, b]}
        return Work([b - a], [0], [a], seed, SYNTH_RANDOM, info,
                    "weak" if world == 1 else "strong")
    # c4 / c5: the commit as pachd serializes it, whole filesets per rank
    sizes = [C4_FILE_BYTES] * C4_FILES
    sizes[-1] += C4_TAIL
    lay = pd.commit_layout(sizes, args.mem_threshold)
    fs = pd.shard_filesets(lay, world)[rank]
    p0, p1 = pd.rank_pieces(lay, fs)
    mode = SYNTH_RANDOM
    if args.config == "c5":
        mode = SYNTH_DEDUP_BLOCKS if args.dedup == "blocks" else SYNTH_DEDUP_FILES
    seed = (0xC4 if args.config == "c4" else 0xC5) if args.seed < 0 else args.seed
    psz = lay.size[p0:p1]
    nbytes = int(psz.sum())
    chains = int(np.sum(np.where(psz > 0, psz // 8_400_000 + 1, 0)))  # ~8.4 MB mean segment
    G = args.group if args.group > 0 else auto_group(chains, nbytes)
    what = "100 GiB" if args.config == "c4" else "100 GiB dedup-heavy (%s)" % args.dedup
    info = {"workload": "configs[%d]: %s commit of %d files (%d B each, +%d on the last), cut "
                        "into serialized filesets of %d B (UnorderedWriter), whole filesets "
                        "per GPU over %d GPU(s); %d commit(s) per step per GPU"
                        % (3 if args.config == "c4" else 4, what, C4_FILES, C4_FILE_BYTES,
                           C4_TAIL, args.mem_threshold, world, G),
            "filesets": lay.nfilesets, "filesets_this_rank": fs[1] - fs[0],
            "pieces_per_commit": lay.npieces, "files_per_step": (p1 - p0) * G,
            "commits_per_step": G, "files_total": C4_FILES}
    if args.config == "c5":
        info["dedup"] = ("1 MiB blocks, p=1/2 a copy of one of 64 pooled blocks"
                         if args.dedup == "blocks" else
                         "whole files, p=1/2 a copy of one of 64 pooled files")
    # copy g of the commit: the same layout over files g * 10000 + f (its own bytes)
    ids = np.concatenate([lay.file[p0:p1].astype(np.int64) + g * C4_FILES for g in range(G)])
    starts = np.tile(lay.start[p0:p1], G)
    w = Work(np.tile(psz, G), ids, starts, seed, mode, info, "strong" if G == 1 else "weak",
             gbase=p0, group=G, per_copy=p1 - p0)
    w.gid = np.concatenate([np.arange(p0, p1, dtype=np.uint64) + np.uint64(g * lay.npieces)
                            for g in range(G)]) if p1 > p0 else w.gid
    w.layout, w.fs_range = lay, fs
    return w


def fill(chunker, tensor, work):
    chunker.fill_synthetic_pieces(tensor, work.offs, work.ids, work.starts, work.seed, work.mode)


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


def host_threads() -> int:
    """Host threads for the CPU baseline: the box's share (OMP_NUM_THREADS, 16 per GPU on the
    GPU pool), else the affinity mask."""
    aff = len(os.sched_getaffinity(0))
    try:
        omp = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        omp = 0
    return min(omp, aff) if omp > 0 else aff


def cpu_model() -> str:
    import platform
    m = platform.processor() or ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return m


def load_traffic(args, work):
    """Per-launch PMC figures (FETCH_SIZE bytes, SQ_INSTS_VALU) of this exact workload."""
    path = args.traffic_json
    if not path and args.config == "c2" and work.group == 32 and args.files == 1024 \
            and args.file_bytes == 4 << 20 and args.path == "put" and not args.ref_ids:
        path = os.path.join(ROOT, "profiles", "r4", "traffic_c2.json")
    if path and os.path.exists(path):
        tj = json.load(open(path))
        tj["_source"] = os.path.relpath(path, ROOT)
        return tj
    return None


def med(xs):
    return round(statistics.median(xs), 4) if xs else None


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
    ``at_least`` (8; 32 for c3's twelve streams) before the first HIP call; a larger setting
    is kept.  The effective value goes into the line's config."""
    try:
        q = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
    except ValueError:
        q = 0
    if q < at_least:
        os.environ["GPU_MAX_HW_QUEUES"] = str(at_least)
        q = at_least
    return q


C3_INFLIGHT, C3_QUEUES, C3_SCAN_GRID = 12, 32, 64
LITERAL_INFLIGHT = 12  # configs1_literal: batches in flight (c2 lines take C3_QUEUES queues)


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
        # a step's scan takes one workgroup per CU; with up to twelve chain-bound hash launches
        # of the other streams holding CUs, capped workgroups never wait for them (the
        # PFSCDC_SCAN_GRID knob, read from the environment when the library first uses a knob;
        # an explicit setting is kept)
        os.environ.setdefault("PFSCDC_SCAN_GRID", str(C3_SCAN_GRID))

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
    cdev = None if rehearse else dev  # collectives' tensors: device (RCCL) or host (gloo)
    ctx = {"np": np, "torch": torch, "dist": dist, "dev": dev, "cdev": cdev, "world": world,
           "rank": rank, "local": local, "pd": pd, "hwq": hwq}

    params = ChunkParams()  # reference defaults: avgBits 23, seed 1, min 1 MB, max 20 MB
    ctx["params"] = params
    if args.path == "uw":
        return bench_uw(args, ctx)
    if args.path == "rechunk":
        return bench_rechunk(args, ctx)
    if args.path == "commit":
        return bench_commit(args, ctx)
    if args.config == "c3" and world > 1 and args.path == "put":
        return bench_c3_split(args, ctx)

    if args.shard:
        sr, sn = (int(x) for x in args.shard.split("/"))
        work = workload(args, sn, sr)
        work.info["shard"] = "rank %d of %d, alone on one GPU" % (sr, sn)
    else:
        work = workload(args, world, rank)
    total = work.total

    # One step at a time by default, so every kernel launch has the GPU to itself and its
    # duration (HIP events, in-kernel span and a kernel trace alike) is its own.  c3 (one
    # stream, bound by its longest 20 MB chains: ~175 ms per stream whatever else runs) runs
    # twelve steps in flight on twelve contexts with 32 hardware queues and scans capped at
    # 64 workgroups (212 GiB/s at four on 8 queues -> 500-547, profiles/r4/c3_queues/);
    # c4/c5 two (the next commit's scan and hashes fill what the chain-bound hash leaves:
    # 824 -> 936 / 820 -> 883 GiB/s, profiles/r3/c4_inflight/);
    # c2's two-in-flight throughput is measured after the timed region (``two_in_flight``).
    # c4/c5 hold >= 16K chains per step through --group instead.
    S = args.inflight if args.inflight > 0 else (
        C3_INFLIGHT if args.path == "put" and args.config == "c3" else
        2 if args.path == "put" and args.config in ("c4", "c5") else 1)
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
    value = float(bytes_step) * args.steps / elapsed / GIB
    ms_per_step = elapsed * 1e3 / K
    intervals = [(b - a) * 1e3 for a, b in zip([t0] + done_at[:-1], done_at)]
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
    try:
        rolled = chunkers[0].last_scan_bytes()
    except Exception:  # noqa: BLE001 - a path without a batch scan
        rolled = total
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

    from pfs_amd import _lib

    info = dict(work.info)
    if c3s:
        info["scan_grid"] = _lib.get_knob("PFSCDC_SCAN_GRID")
    try:
        smode = chunkers[0].last_scan_mode()
    except Exception:  # noqa: BLE001 - a path without a batch scan
        smode = 0
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
    out = {
        "metric": "GiB/s device-resident CDC rolling-hash + chunk content-hash",
        "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
        "scaling": work.scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 bytes generated in HBM)",
        "ref_ids": bool(args.ref_ids),
        "config": info,
        "segments_per_step": int(len(res.segments)),
        "ms_per_step_median": med(intervals),
        "kernel_ms": kmean,
        "kernel_ms_median": kmed,
        "note": "kernel_ms: per step on this rank; scan/select/hash = HIP events on the "
                "library's stream (with steps in flight they include waiting for CUs behind "
                "the other step), scan_span/hash_span = the kernels' own execution spans "
                "(first wavefront start to last wavefront end); the hash is VALU-issue bound, "
                "not HBM bound (DESIGN.md §4)",
        "cdc_only_gib_s": round(total / (scan_ms * 1e-3) / GIB, 2) if scan_ms else None,
        "hash_only_gib_s": round(total / (hash_ms * 1e-3) / GIB, 2) if hash_ms else None,
        "roofline": roofline,
        "roofline_cdc": roofline_cdc,
    }
    if rvalu:
        out["roofline_valu"] = rvalu
    if S > 1:
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
        out["single_commit"] = single_commit(args, work, chunkers[0], batches[0], ctx)
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
        out["index_digest"] = __import__("hashlib").blake2b(idx.tobytes(),
                                                            digest_size=16).hexdigest()
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

    if rank == 0 and world == 1 and not args.no_chain_floor:
        out["chain_floor"] = chain_floor(res, hash_ms, data, params, local, Chunker)
    if rank == 0 and world == 1 and args.config == "c2" and S == 1 and not args.no_pipelined:
        out["two_in_flight"] = two_in_flight(args, work, chunker, data, params, local, Chunker,
                                             torch)
    if rank == 0 and world == 1 and args.config == "c2" and not args.no_literal:
        out["configs1_literal"] = literal_batch(args, work, chunker, data, params, local,
                                                Chunker, torch)
    if rank == 0 and world == 1 and args.config == "c2" and not args.no_e2e:
        out["e2e"] = e2e(args, work, data, params, local, Chunker, torch, np)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_baseline(args, work, data, res, params, out, np, last)

    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    chunker.close()


def single_commit(args, work, chunker, data, ctx):
    """One commit per step (G = 1) on the same ranks and contexts: the step time of the
    configured 100 GiB commit itself over N GPUs (strong scaling), max over ranks."""
    torch, dist, world, cdev = ctx["torch"], ctx["dist"], ctx["world"], ctx["cdev"]
    offs0 = work.offs[:work.per_copy + 1]
    total0 = int(offs0[-1])
    part = data[:total0]
    for _ in range(max(1, args.warmup)):
        chunker.scan_async(part, offs0)
        chunker.wait()
    k = max(2, min(args.steps, 4))
    hs = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        chunker.scan_async(part, offs0)
        chunker.wait()
        hs.append(chunker.timings()["hash_span"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    nb = float(total0)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        bt = torch.tensor([nb], dtype=torch.float64, device=cdev)
        dist.all_reduce(bt, op=dist.ReduceOp.SUM)
        nb = float(bt.item())
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


def two_in_flight(args, work, chunker, data, params, local, Chunker, torch):
    """After the timed region: the same steps with two in flight (a second context on its own
    stream over its own copy of the input), so the next step's scan fills the CUs this step's
    hash frees as its queue drains.  Reported beside the contract's one-at-a-time value."""
    try:
        data2 = torch.empty_like(data)
    except torch.OutOfMemoryError:
        return {"skipped": "HBM cannot hold a second input"}
    data2.copy_(data)
    other = Chunker(params, device=local)
    pair, bufs, busy = [chunker, other], [data, data2], [False, False]
    n, warm = 10, 2
    t0 = None
    for i in range(warm + n):
        if i == warm:
            for k in range(2):
                if busy[k]:
                    pair[k].wait()
                    busy[k] = False
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        k = i % 2
        if busy[k]:
            pair[k].wait()
        pair[k].scan_async(bufs[k], work.offs)
        busy[k] = True
    for j in range(2):
        k = (warm + n + j) % 2
        if busy[k]:
            pair[k].wait()
    el = time.perf_counter() - t0
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
    pair = [chunker, other]
    busy = [False, False]
    other.scan(view, offs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps * 2):
        k = i % 2
        if busy[k]:
            pair[k].wait()
        pair[k].scan_async(view, offs)
        busy[k] = True
    for k in range(2):
        if busy[(reps * 2 + k) % 2]:
            pair[(reps * 2 + k) % 2].wait()
    piped = (time.perf_counter() - t0) / (reps * 2)
    other.close()
    # many batches in flight: LITERAL_INFLIGHT contexts (one stream and hardware queue each),
    # every call still one configs[1] batch; the batches' ~4 MiB chains overlap instead of
    # aggregating into one launch
    k = LITERAL_INFLIGHT
    many = [chunker] + [Chunker(params, device=local) for _ in range(k - 1)]
    for c in many[1:]:
        c.scan(view, offs)
    torch.cuda.synchronize()
    busy = [False] * k
    nmany = 4 * k
    t0 = time.perf_counter()
    for i in range(nmany):
        j = i % k
        if busy[j]:
            many[j].wait()
        many[j].scan_async(view, offs)
        busy[j] = True
    for j in range(k):
        if busy[j]:
            many[j].wait()
    piped_k = (time.perf_counter() - t0) / nmany
    for c in many[1:]:
        c.close()
    return {"value": round(sb / serial / GIB, 3), "unit": "GiB/s",
            "ms_per_batch": round(serial * 1e3, 3),
            "hash_span_ms_median": round(statistics.median(hs), 3),
            "two_in_flight_value": round(sb / piped / GIB, 3),
            "many_in_flight": {"batches_in_flight": k, "value": round(sb / piped_k / GIB, 3),
                               "ms_per_batch": round(piped_k * 1e3, 3),
                               "note": "%d contexts on %d streams, one configs[1] batch per "
                                       "call, %d batches" % (k, k, nmany)},
            "note": "one configs[1] batch (1024 x 4 MiB) per step, device-resident, no "
                    "aggregation: bound by the ~4 MiB serial BLAKE2b chains (DESIGN.md §4)"}


def e2e(args, work, data, params, local, Chunker, torch, np):
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


def cpu_baseline(args, work, data, res, params, out, np, last):
    """The C restatement of the reference chunker (oracle, kind "port") on the host threads
    the box allots, over a bounded sample of the same workload, plus the parity check of the
    GPU records on that sample."""
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
    p = och.Params(params.average_bits, params.seed, params.min_chunk, params.max_chunk)
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


def bench_c3_split(args, ctx):
    """configs[2] on N GPUs: one 10 GiB stream in equal byte ranges (strong scaling).  A step =
    candidates of the rank's range (+64-byte halo), all-gather of the candidates, the serial
    selection, point-to-point copies of straddling segments' bytes, BLAKE2b of the segments
    starting in the range, all-gather of the segment records."""
    np, torch, dist, pd = ctx["np"], ctx["torch"], ctx["dist"], ctx["pd"]
    from pfs_amd.cdc import Chunker, SYNTH_RANDOM

    world, rank, dev, cdev, params = ctx["world"], ctx["rank"], ctx["dev"], ctx["cdev"], ctx["params"]
    seed = 0xC3 if args.seed < 0 else args.seed
    n = C3_BYTES
    a, b = pd.split_stream(n, world)[rank]
    halo = min(a, 64)
    local = torch.zeros(halo + (b - a) + params.max_chunk, dtype=torch.uint8, device=dev)
    ch = Chunker(params, device=ctx["local"])
    ch.fill_synthetic_pieces(local[:halo + b - a], [0, halo + b - a], [0], [a - halo], seed,
                             SYNTH_RANDOM)
    # collectives over RCCL on device tensors (gloo on host tensors when rehearsing)
    cand_fn = (lambda t, h: ch.candidates(t, h))
    hash_fn = (lambda t, bb, zz: ch.hash_ranges(t, bb, zz))
    split = {"cand_ms": [], "hash_ms": [], "step_ms": []}

    def step(record):
        t0 = time.perf_counter()
        segs = pd.stream_segments(local, n, (a, b), halo, params.min_chunk, params.max_chunk,
                                  cand_fn, hash_fn, device=cdev)
        if record:
            tm = ch.timings()
            split["cand_ms"].append(tm["scan"])
            split["hash_ms"].append(tm["hash"])
            split["step_ms"].append((time.perf_counter() - t0) * 1e3)
        return segs

    for _ in range(args.warmup):
        step(False)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        segs = step(True)
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    K = max(args.steps, 1)
    info = workload(args, world, rank).info
    info.update({"parallelism": "stream split x%d: candidates all-gather, serial select, "
                                "RCCL send/recv of border segments, records all-gather" % world})
    out = {
        "metric": "GiB/s device-resident CDC rolling-hash + chunk content-hash",
        "value": round(n * args.steps / elapsed / GIB, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / K, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 bytes generated in HBM)", "config": info,
        "ms_median": {k: med(v) for k, v in split.items()},
        "index_digest": __import__("hashlib").blake2b(segs.tobytes(), digest_size=16).hexdigest(),
        "index_segments": int(len(segs)),
        "note": "hash_ms: this rank's segments (a split stream is bound by its longest serial "
                "BLAKE2b chains, up to max = 20 MB)",
    }
    if rank == 0:
        print(json.dumps(out))
    dist.destroy_process_group()
    ch.close()


def bench_get(args, ctx, chunker, data, work):
    """Read path: the step's segments are stored chunks (chunk.Create form); one step =
    pfscdc_get_chunks over all of them (verify + decrypt, device in/out)."""
    np, torch, dist = ctx["np"], ctx["torch"], ctx["dist"]
    world, rank, cdev = ctx["world"], ctx["rank"], ctx["cdev"]
    total, offs = work.total, work.offs
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
    kms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        _, ok = chunker.get_chunks(ctext, cofs, res.refs, out=out)
        kms.append(chunker.last_get_ms())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    same = bool(ok.all()) and bool(torch.equal(out, data))
    bytes_step = total
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        bt = torch.tensor([total], dtype=torch.float64, device=cdev)
        dist.all_reduce(bt, op=dist.ReduceOp.SUM)
        bytes_step = int(bt.item())
    K = max(args.steps, 1)
    ms = sum(kms) / len(kms) if kms else 0.0
    ach = total / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    info = dict(work.info)
    info.update({"path": "get (chunk.Get: verify Ref.Id, ChaCha20 decrypt)",
                 "chunks_per_step": int(len(segs))})
    out_line = {
        "metric": "GiB/s device-resident chunk.Get (verify + decrypt) of stored chunks",
        "value": round(float(bytes_step) * args.steps / elapsed / GIB, 3), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / K, 3), "higher_is_better": True,
        "scaling": work.scaling, "vs_baseline": None, "dtype": "u8",
        "data": "synthetic plaintext encrypted on the GPU with its own Ref.Dek", "config": info,
        "kernel_ms": {"get": round(ms, 4)}, "kernel_ms_median": {"get": med(kms)},
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
    """(piece sizes, fileset begin indices over pieces) of UnorderedWriter.Put of the files in
    path order: pfs_amd.distributed.commit_layout (unordered_writer.go:45-72)."""
    from pfs_amd import distributed as pd
    lay = pd.commit_layout(sizes, mem_threshold)
    return [int(x) for x in lay.size], [int(x) for x in lay.fileset_begin]


def bench_commit(args, ctx):
    """pachd data plane on the step's files: pieces / filesets (commit_layout), CDC + DataRef
    hashes (one scan of all pieces), chunk formation per fileset stream (pfscdc_form_chunks),
    chunk.Create of every formed chunk (pfscdc_create_refs: content hash of multi-DataRef
    chunks, dek, ChaCha20 + BLAKE2b of the ciphertext).

    N>1: whole serialized filesets per rank (a fresh chunk.Writer per fileset, so chunks never
    span ranks); each rank forms its chunks and Refs, and the chunk records (offset in the
    commit stream, size, Ref.Id, Ref.Dek) are all-gathered: the same list as N=1.

    With --inflight S > 1, S contexts (S HIP streams) each run every S-th step from their own
    host thread, so one step's chunk.Create tail (the serial BLAKE2b chains of its largest
    chunks: content hash, then Ref.Id) overlaps the next step's scan and hashes.  The steps
    read the same device buffer (the same files committed again; the library only reads it)."""
    import threading

    np, torch, dist, pd = ctx["np"], ctx["torch"], ctx["dist"], ctx["pd"]
    world, rank, dev, cdev, params = ctx["world"], ctx["rank"], ctx["dev"], ctx["cdev"], ctx["params"]
    from pfs_amd.cdc import Chunker

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
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        bt = torch.tensor([total], dtype=torch.float64, device=cdev)
        dist.all_reduce(bt, op=dist.ReduceOp.SUM)
        bytes_step = int(bt.item())
    K = max(args.steps, 1)
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
    import hashlib
    metric = ("GiB/s device-resident pachd commit data plane (CDC + DataRef hashes + "
              "chunk formation + chunk.Create Ref.Id)") if not args.no_create else (
              "GiB/s device-resident CDC + every BLAKE2b of Writer.processChunk (DataRef hashes "
              "+ chunk content hashes, writer.go:240,301-312) + chunk formation")
    out = {
        "metric": metric,
        "value": round(float(bytes_step) * args.steps / elapsed / GIB, 3), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / K, 3), "higher_is_better": True,
        "scaling": work.scaling if G > 1 else "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 bytes generated in HBM)", "config": info,
        "kernel_ms": {name: round(v, 4) for name, v in avg.items()},
        "commit_chunks_digest": hashlib.blake2b(chunks.tobytes(), digest_size=16).hexdigest(),
        "dataref_hashes_digest": hashlib.blake2b(dr_hashes.tobytes(), digest_size=16).hexdigest(),
        "roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "traffic": None,
                     "bytes_per_launch": total, "avg_launch_ms": round(ms, 4),
                     "kernel": "chunk.Create batch (content hash + dek + ChaCha20/BLAKE2b)"
                     if not args.no_create else
                     "one BLAKE2b launch over every segment and multi-DataRef chunk"},
    }
    if S > 1:
        out["note"] = ("kernel_ms are per step on its own stream; with %d steps in flight they "
                       "overlap, so ms_per_step < their sum" % S)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if in_place:  # the buffer holds the verification step's ciphertext
            fill(chunkers[0], data, work)
        out["parity"] = commit_parity(data, work, streams, last, params, np)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()
    for ch in chunkers:
        ch.close()


def bench_uw(args, ctx):
    """Host-fed pachd write path: the first --uw-bytes of the commit's files (host memory) Put
    through the UnorderedWriter (pfs_amd.fileset over pfscdc_uw_*): buffering, 1e9-byte
    filesets, GPU chunk writers with Ref ids, index writers.  N>1: whole serialized filesets
    per rank (each rank its own UnorderedWriter over its pieces, the re-Added continuation of
    a split file Put with append); the filesets (SizeBytes, root indexes) are all-gathered:
    the same list as one writer's."""
    np, torch, dist, pd = ctx["np"], ctx["torch"], ctx["dist"], ctx["pd"]
    world, rank, dev, cdev, params = ctx["world"], ctx["rank"], ctx["dev"], ctx["cdev"], ctx["params"]
    from pfs_amd import fileset as pf
    from pfs_amd.cdc import Chunker

    base = workload(args, 1, 0) if args.config in ("c2", "c3") else None
    if base is None:
        sizes = [C4_FILE_BYTES] * C4_FILES
        sizes[-1] += C4_TAIL
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
    from pfs_amd import _lib
    if args.uw_workers > 0:
        _lib.set_knob("PFSCDC_UW_WORKERS", args.uw_workers)
    if args.uw_group > 0:
        _lib.set_knob("PFSCDC_UW_INFLIGHT", args.uw_group)
    st = pf.Storage(ctx["local"], params, args.mem_threshold)

    def step():
        t = time.perf_counter()
        w = st.new_unordered_writer()
        w.create_ms = (time.perf_counter() - t) * 1e3
        prims = pd.put_rank_filesets(w, lay, fs, lambda f: "/%016d" % f,
                                     lambda f, s, n: views[(f, s)])
        tm = w.timings()
        tm["writer_create"] = w.create_ms
        nch = sum(1 for fsv in w.events for e in fsv if e[0] == "chunk" and e[1] == -1)
        w.release()  # its data context goes back to the Storage for the next commit
        return prims, tm, nch

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    stages = {}
    for _ in range(args.steps):
        prims, tm, nchunks = step()
        for k, v in tm.items():
            stages[k] = stages.get(k, 0.0) + v / max(args.steps, 1)
    elapsed = time.perf_counter() - t0
    bytes_step = nbytes
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
        bt = torch.tensor([nbytes], dtype=torch.float64, device=cdev)
        dist.all_reduce(bt, op=dist.ReduceOp.SUM)
        bytes_step = int(bt.item())
    gathered = pd.gather_primitives(prims, device=cdev) if world > 1 else \
        [(p.additive, p.deletive, p.size_bytes) for p in prims]
    import hashlib
    K = max(args.steps, 1)
    info = {"workload": "the first %d files (%d B) of %s, Put from host memory" % (
                nf, int(offs[nf]), args.config),
            "path": "uw (host-fed UnorderedWriter -> fileset.Writer -> index.Writer)",
            "bytes_this_rank": nbytes, "mem_threshold": args.mem_threshold,
            "filesets": lay.nfilesets, "filesets_this_rank": len(prims),
            "data_chunks_this_rank": nchunks, "gpu_max_hw_queues": ctx["hwq"],
            "parallelism": "fileset-sharded x%d, all-gather of the fileset roots" % world
            if world > 1 else "single GPU"}
    out = {
        "metric": "GiB/s host-fed pachd write path (Put -> filesets with chunk Refs and "
                  "multilevel indexes)",
        "value": round(float(bytes_step) * args.steps / elapsed / GIB, 3), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / K, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic bytes in host memory", "config": info,
        "commit_filesets_digest": hashlib.blake2b(
            b"".join(pd.encode_primitive(*g) for g in gathered), digest_size=16).hexdigest(),
        "note": "a step: the Puts (one host copy into the fileset arenas) and the grouped "
                "GPU write of every fileset plus the indexes, then Close",
        "stages_ms": {k: round(v, 2) for k, v in stages.items()},
        "stages_note": "per step; put_copy on the Put thread, the rest summed over the group "
                       "writes (a background thread per group writer, %s writer(s), each on its own ctx), "
                       "so they overlap the Puts and each other (pfscdc_uw_timings)"
                       % _lib.get_knob("PFSCDC_UW_WORKERS"),
    }
    if stages.get("put_copy"):
        out["put_copy_gb_s"] = round(nbytes / (stages["put_copy"] * 1e-3) / 1e9, 2)
        out["host_memcpy_gb_s"] = host_memcpy_rate(torch, min(nbytes, 4 << 30))
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def host_memcpy_rate(torch, nbytes):
    """The ceiling of the Put copy: a large host-to-page-locked copy on the job's threads
    (torch's parallel CPU copy, OMP_NUM_THREADS), best of 3, GB/s."""
    src = torch.empty(nbytes, dtype=torch.uint8).fill_(7)
    dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    best = 0.0
    for _ in range(3):
        t = time.perf_counter()
        dst.copy_(src)
        best = max(best, nbytes / (time.perf_counter() - t) / 1e9)
    return {"gb_s": round(best, 2), "threads": torch.get_num_threads(), "bytes": nbytes}


def bench_rechunk(args, ctx):
    """Re-chunk path (MergeFileReader.Hash, the Writer.Copy machinery): a 1 GiB file written
    by --rechunk-writers writers (each its own chunk stream, ciphertexts uploaded to the
    in-memory store), then the merged file's hash: Copy of every DataRef through a fresh
    writer, whole aligned chunks passed through, the rest read back (chunk.Get on the GPU) and
    re-rolled.  Checked against the single-writer hash."""
    np, torch, dev = ctx["np"], ctx["torch"], ctx["dev"]
    world = ctx["world"]
    from pfs_amd import chunk as pc
    from pfs_amd.cdc import Chunker, SYNTH_RANDOM

    nbytes = 1 << 30
    gen = Chunker(ctx["params"], device=ctx["local"])
    t = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    gen.fill_synthetic(t, [0, nbytes], 0xC2 if args.seed < 0 else args.seed, SYNTH_RANDOM)
    host = t.cpu().numpy()
    gen.close()
    del t
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
    info = {"path": "rechunk (MergeFileReader.Hash of a file written by %d writers)" % k,
            "file_bytes": nbytes, "data_refs": len(refs), "edge_data_refs": edge,
            "store_chunks": len(store)}
    out = {
        "metric": "GiB/s of file bytes through MergeFileReader.Hash (Writer.Copy re-chunking)",
        "value": round(nbytes * args.steps / elapsed / GIB, 3), "unit": "GiB/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / K, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded splitmix64 bytes generated in HBM, copied to host)",
        "config": info,
        "parity": {"merged_hash_equals_single_writer_hash": got == want},
    }
    if ctx["rank"] == 0:
        print(json.dumps(out))
    if world > 1:
        ctx["dist"].destroy_process_group()


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
        import hashlib
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


if __name__ == "__main__":
    main()
