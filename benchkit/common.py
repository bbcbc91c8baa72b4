"""Shared pieces of the benchmark legs: constants, the synthetic workloads of BASELINE.json's
configs, and small helpers.  No leg-specific timing here (harness.py owns the timing rule)."""
import json
import math
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

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
C3_INFLIGHT, C3_QUEUES, C3_SCAN_GRID = 20, 32, 64
LITERAL_INFLIGHT = 20  # configs1_literal: batches in flight (c2 lines take C3_QUEUES queues)
METRIC = "GiB/s device-resident CDC rolling-hash + chunk content-hash"
SYNTH_DATA = "synthetic (seeded splitmix64 bytes generated in HBM)"


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


def c4_sizes():
    sizes = [C4_FILE_BYTES] * C4_FILES
    sizes[-1] += C4_TAIL
    return sizes


def workload(args, world, rank):
    """This rank's pieces for one step."""
    import numpy as np

    from pfs_amd import distributed as pd
    from pfs_amd.cdc import SYNTH_DEDUP_BLOCKS, SYNTH_DEDUP_FILES, SYNTH_RANDOM

    if args.config == "c2":
        # the read path holds three copies of the step (stored, ciphertext, decrypted): 16
        # batches (3 x 64 GiB) fit in HBM, 32 do not
        G = args.group if args.group > 0 else (16 if args.path == "get" else 32)
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
    lay = pd.commit_layout(c4_sizes(), args.mem_threshold)
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


def commit_layout(sizes, mem_threshold):
    """(piece sizes, fileset begin indices over pieces) of UnorderedWriter.Put of the files in
    path order: pfs_amd.distributed.commit_layout (unordered_writer.go:45-72)."""
    from pfs_amd import distributed as pd
    lay = pd.commit_layout(sizes, mem_threshold)
    return [int(x) for x in lay.size], [int(x) for x in lay.fileset_begin]


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
        path = os.path.join(ROOT, "profiles", "r6", "final", "traffic_c2.json")
    if path and os.path.exists(path):
        tj = json.load(open(path))
        tj["_source"] = os.path.relpath(path, ROOT)
        return tj
    return None


def med(xs):
    return round(statistics.median(xs), 4) if xs else None


def host_memcpy_rate(torch, nbytes):
    """The ceiling of the Put copy: a large host-to-page-locked copy on the job's threads
    (torch's parallel CPU copy, OMP_NUM_THREADS), best of 3, GB/s."""
    import time
    src = torch.empty(nbytes, dtype=torch.uint8).fill_(7)
    dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    best = 0.0
    for _ in range(3):
        t = time.perf_counter()
        dst.copy_(src)
        best = max(best, nbytes / (time.perf_counter() - t) / 1e9)
    return {"gb_s": round(best, 2), "threads": torch.get_num_threads(), "bytes": nbytes}
