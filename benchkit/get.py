"""Read path (chunk.Get, transform.go:50-78): the step's segments are stored chunks (the
chunk.Create form); one step = pfscdc_get_chunks over all of them (verify BLAKE2b of the
stored bytes against Ref.Id, ChaCha20 decrypt), device-resident in and out."""
from .common import HBM_PEAK_GBS, med
from .harness import Harness


def bench_get(args, ctx, chunker, data, work):
    np, torch = ctx["np"], ctx["torch"]
    H = Harness(ctx)
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
    kms, last = [], {}

    def run(k):
        for _ in range(k):
            _, last["ok"] = chunker.get_chunks(ctext, cofs, res.refs, out=out)
            kms.append(chunker.last_get_ms())

    elapsed = H.timed(run, args.steps)
    ok = last["ok"]
    same = bool(ok.all()) and bool(torch.equal(out, data))
    bytes_step = H.sum_over_ranks(total)
    ms = sum(kms) / len(kms) if kms else 0.0
    ach = total / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    info = dict(work.info)
    info.update({"path": "get (chunk.Get: verify Ref.Id, ChaCha20 decrypt)",
                 "chunks_per_step": int(len(segs))})
    line = H.line("GiB/s device-resident chunk.Get (verify + decrypt) of stored chunks",
                  bytes_step, args.steps, args.warmup, elapsed, work.scaling, info,
                  data="synthetic plaintext encrypted on the GPU with its own Ref.Dek",
                  kernel_ms={"get": round(ms, 4)}, kernel_ms_median={"get": med(kms)},
                  roofline={"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5),
                            "traffic": None, "bytes_per_launch": total,
                            "avg_launch_ms": round(ms, 4), "kernel": "blake2b_kernel<kModeGet>"},
                  parity={"all_chunks_verified": bool(ok.all()),
                          "plaintext_equals_original": same})
    H.emit(line)
    H.close()
    chunker.close()
