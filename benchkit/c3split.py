"""configs[2] on N GPUs: one 10 GiB stream in equal byte ranges (strong scaling).  A step =
candidates of the rank's range (+64-byte halo), all-gather of the candidates, the serial
selection, point-to-point copies of straddling segments' bytes, BLAKE2b of the segments
starting in the range, all-gather of the segment records (pfs_amd.distributed.stream_segments).
"""
import hashlib
import time

from . import parity as par
from .common import C3_BYTES, METRIC, med, workload
from .harness import Harness


def bench_c3_split(args, ctx):
    torch, pd = ctx["torch"], ctx["pd"]
    from pfs_amd.cdc import Chunker, SYNTH_RANDOM

    H = Harness(ctx)
    world, rank, dev, cdev, params = ctx["world"], ctx["rank"], ctx["dev"], ctx["cdev"], ctx["params"]
    seed = 0xC3 if args.seed < 0 else args.seed
    n = C3_BYTES
    ranges = pd.split_stream(n, world)
    a, b = ranges[rank]
    halo = min(a, 64)
    local = torch.zeros(halo + (b - a) + params.max_chunk, dtype=torch.uint8, device=dev)
    ch = Chunker(params, device=ctx["local"])
    ch.fill_synthetic_pieces(local[:halo + b - a], [0, halo + b - a], [0], [a - halo], seed,
                             SYNTH_RANDOM)
    # collectives over RCCL on device tensors (gloo on host tensors when rehearsing)
    cand_fn = (lambda t, h: ch.candidates(t, h))
    hash_fn = (lambda t, bb, zz: ch.hash_ranges(t, bb, zz))
    split = {"cand_ms": [], "hash_ms": [], "step_ms": []}
    last = {}

    def step(record):
        t0 = time.perf_counter()
        last["segs"] = pd.stream_segments(local, n, (a, b), halo, params.min_chunk,
                                          params.max_chunk, cand_fn, hash_fn, device=cdev)
        if record:
            tm = ch.timings()
            split["cand_ms"].append(tm["scan"])
            split["hash_ms"].append(tm["hash"])
            split["step_ms"].append((time.perf_counter() - t0) * 1e3)

    def run(k):
        for _ in range(k):
            step(True)

    for _ in range(args.warmup):
        step(False)
    elapsed = H.timed(run, args.steps)
    segs = last["segs"]
    info = workload(args, world, rank).info
    info.update({"parallelism": "stream split x%d: candidates all-gather, serial select, "
                                "RCCL send/recv of border segments, records all-gather" % world})
    out = H.line(METRIC, n, args.steps, args.warmup, elapsed, "strong", info,
                 ms_median={k: med(v) for k, v in split.items()},
                 index_digest=hashlib.blake2b(segs.tobytes(), digest_size=16).hexdigest(),
                 index_segments=int(len(segs)),
                 note="hash_ms: this rank's segments (a split stream is bound by its longest "
                      "serial BLAKE2b chains, up to max = 20 MB)")
    if rank == 0:
        out["parity"] = par.stream_border_parity(segs, n, ranges, seed, params)
    H.emit(out)
    H.close()
    ch.close()
