"""Re-chunk path (--path rechunk: MergeFileReader.Hash, the Writer.Copy machinery,
fileset/merge.go:125-143, chunk/writer.go:315-420): a 1 GiB file written by
--rechunk-writers writers (each its own chunk stream, ciphertexts uploaded to the in-memory
store), then the merged file's hash: Copy of every DataRef through a fresh writer, whole
aligned chunks passed through, the rest read back (chunk.Get on the GPU) and re-rolled.
Checked against the single-writer hash (the reference's TestStableHash property)."""
from .harness import Harness


def bench_rechunk(args, ctx):
    torch, dev = ctx["torch"], ctx["dev"]
    from pfs_amd import chunk as pc
    from pfs_amd.cdc import Chunker, SYNTH_RANDOM

    H = Harness(ctx)
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
    last = {}

    def run(n):
        for _ in range(n):
            last["got"] = pc.merge_file_hash(store, refs, device=dev.index or 0)

    elapsed = H.timed(run, args.steps)
    edge = sum(1 for d in refs if d.ref.edge)
    info = {"path": "rechunk (MergeFileReader.Hash of a file written by %d writers)" % k,
            "file_bytes": nbytes, "data_refs": len(refs), "edge_data_refs": edge,
            "store_chunks": len(store)}
    out = H.line("GiB/s of file bytes through MergeFileReader.Hash (Writer.Copy re-chunking)",
                 H.sum_over_ranks(nbytes), args.steps, args.warmup, elapsed, "weak", info,
                 data="synthetic (seeded splitmix64 bytes generated in HBM, copied to host)",
                 parity={"merged_hash_equals_single_writer_hash": last.get("got") == want})
    H.emit(out)
    H.close()
