#!/usr/bin/env python3
"""Generates tests/golden/golden.json from the Python oracle (oracle/chunker.py).

Run from the repo root:  python tests/golden/make_golden.py
Inputs are described, not stored: the synthetic byte stream (pfs_amd.cdc.synthetic_bytes,
also the device generator) with the seeds and offsets recorded in each case.  The small
cases are produced by the literal byte-by-byte Writer, the large ones by the numpy closed
form (both cross-checked in tests/test_oracle_consistency.py).

Provenance: these vectors come from our restatement of the reference chunker, pinned by the
known-answer tests in tests/test_oracle_kat.py; no Go toolchain was available to produce
them from the reference itself, so they anchor regressions, not parity with
a Go run.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import buzhash64, chunker as Ch, gorand  # noqa: E402
from pfs_amd.cdc import synthetic_bytes  # noqa: E402


def seg_case(name, params, offs, seed, segmenter):
    data = synthetic_bytes(offs, seed)
    files = [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(len(offs) - 1)]
    chunks = Ch.chunk_stream(files, params, segmenter=segmenter)
    per_file = Ch.file_segments_from_chunks(chunks, len(files))
    cut_info = [Ch.segments_numpy(f, params) if segmenter == "numpy" else Ch.segments_literal(f, params)
                for f in files]
    segs = []
    for f in range(len(files)):
        assert [(o, s) for o, s, _ in per_file[f]] == [(o, s) for o, s, _ in cut_info[f]]
        for (o, s, h), (_, _, cut) in zip(per_file[f], cut_info[f]):
            segs.append([f, o, s, int(cut), h.hex()])
    chunk_list = []
    for c in chunks:
        refs = [[a.data, a.next_data_ref.offset_bytes, a.next_data_ref.size_bytes,
                 a.next_data_ref.hash.hex()] for a in c.annotations if a.next_data_ref]
        chunk_list.append([len(c.data), int(c.edge), refs])
    return {"name": name,
            "params": {"average_bits": params.average_bits, "seed": params.seed,
                       "min": params.min, "max": params.max},
            "data": {"generator": "synthetic_bytes", "seed": seed,
                     "file_offsets": [int(x) for x in offs]},
            "segments": segs,
            "chunks": chunk_list,
            "file_hashes": [Ch.file_hash([h for _, _, h in per_file[f]]).hex()
                            for f in range(len(files))]}


def main():
    out = {"tables": {}, "go_int63": {}, "cases": []}
    for s in (0, 1, 2):
        out["tables"][str(s)] = ["%016x" % x for x in buzhash64.generate_hashes(s)]
    for s in (0, 1, 2, 42, -1):
        src = gorand.Source(s)
        out["go_int63"][str(s)] = [src.int63() for _ in range(8)]

    rng = np.random.default_rng(1)
    lens = rng.integers(0, 50_000, 60)
    lens[::9] = 0
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    small = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
    out["cases"].append(seg_case("small_multi_literal", small, offs, 1, "literal"))

    offs = np.arange(9, dtype=np.uint64) * np.uint64(4 << 20)
    out["cases"].append(seg_case("c2_mini_8x4MiB", Ch.Params(), offs, 0xC2, "numpy"))

    offs = np.array([0, 64 << 20], dtype=np.uint64)
    out["cases"].append(seg_case("stream_64MiB", Ch.Params(), offs, 0xC3, "numpy"))

    rng = np.random.default_rng(4)
    lens = rng.integers(0, 3_000_000, 24)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    out["cases"].append(seg_case("multi_file_chunks_default", Ch.Params(), offs, 0xC4, "numpy"))

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
