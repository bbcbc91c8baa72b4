"""Golden fixtures (tests/golden/golden.json, made by tests/golden/make_golden.py).

CPU: the C oracle and the product's native table generator reproduce the fixtures.
GPU: the HIP path reproduces every segment, digest and FileInfo hash of every case.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import chunker as Ch
from oracle import coracle
from pfs_amd import _lib
from pfs_amd.cdc import synthetic_bytes

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def case_inputs(case):
    p = case["params"]
    params = Ch.Params(p["average_bits"], p["seed"], p["min"], p["max"])
    offs = np.asarray(case["data"]["file_offsets"], dtype=np.uint64)
    data = synthetic_bytes(offs, case["data"]["seed"])
    return params, offs, data


def golden_rows(case):
    return [(f, o, s, c, h) for f, o, s, c, h in case["segments"]]


def rows_from(segs):
    return [(int(s["file"]), int(s["offset"]), int(s["size"]), int(bool(s["flags"] & 2)),
             bytes(s["hash"]).hex()) for s in segs]


def test_product_tables_match_golden():
    for seed, hexes in GOLDEN["tables"].items():
        assert ["%016x" % x for x in _lib.table(int(seed))] == hexes


def test_product_go_rand_matches_golden():
    for seed, vals in GOLDEN["go_int63"].items():
        assert _lib.go_int63(int(seed), len(vals)) == vals


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=[c["name"] for c in GOLDEN["cases"]])
def test_c_oracle_matches_golden(case):
    params, offs, data = case_inputs(case)
    segs, _ = coracle.segment_files(data, offs, params, nthreads=4)
    assert rows_from(segs) == golden_rows(case)


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=[c["name"] for c in GOLDEN["cases"]])
def test_file_hashes_golden(case):
    per_file = [[] for _ in range(len(case["data"]["file_offsets"]) - 1)]
    for f, _, _, _, h in case["segments"]:
        per_file[f].append(bytes.fromhex(h))
    got = [Ch.file_hash(x).hex() for x in per_file]
    assert got == case["file_hashes"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", GOLDEN["cases"], ids=[c["name"] for c in GOLDEN["cases"]])
def test_gpu_matches_golden(case):
    from pfs_amd.cdc import ChunkParams, Chunker

    params, offs, data = case_inputs(case)
    c = Chunker(ChunkParams(params.average_bits, params.seed, params.min, params.max), 0)
    res = c.scan(data, offs)
    assert rows_from(res.segments) == golden_rows(case)
    # FileInfo.Hash = BLAKE2b(concat DataRef.Hash) (fileset/util.go:149-158)
    for f, want in enumerate(case["file_hashes"]):
        h = hashlib.blake2b(digest_size=32)
        for s in res.file_segments(f):
            h.update(bytes(s["hash"]))
        assert h.hexdigest() == want
    c.close()
