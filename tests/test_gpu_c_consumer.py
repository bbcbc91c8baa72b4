"""GPU parity from a plain C process: tests/c/abi_gpu_consumer.c includes only pfscdc.h and
links -lpfscdc, as a cgo binary in pachd would, with no Python or torch in the process.  It
scans a batch with Ref ids and runs the chunk.Writer mirror over the same files; every line
it prints is checked against the oracle over the bytes it wrote out."""
import os
import subprocess

import numpy as np
import pytest

from conftest import fuzz_cases

from oracle import chunker as Ch
from oracle import coracle
from pfs_amd import _lib

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def consumer(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("c") / "abi_gpu_consumer")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "abi_gpu_consumer.c"),
                    "-L", libdir, "-lpfscdc", "-Wl,-rpath," + libdir,
                    "-Wl,-rpath-link,/opt/rocm/lib", "-o", exe], check=True)
    return exe


def run(consumer, tmp_path, p, batch_bytes, lens):
    data_path = str(tmp_path / "data.bin")
    res = subprocess.run([consumer, data_path, str(p.average_bits), str(p.seed), str(p.min),
                          str(p.max), str(batch_bytes)] + [str(int(x)) for x in lens],
                         capture_output=True, text=True, timeout=100)
    assert res.returncode == 0, res.stderr
    data = np.fromfile(data_path, dtype=np.uint8)
    assert len(data) == int(sum(lens))
    return res.stdout.splitlines(), data


@pytest.mark.parametrize("case", fuzz_cases(3))
def test_c_process_scan_and_writer_equal_oracle(consumer, tmp_path, case):
    rng = np.random.default_rng(4200 + case)
    p = [Ch.Params(average_bits=12, seed=1, min=2000, max=30000),
         Ch.Params(average_bits=10, seed=int(rng.integers(0, 5)), min=64, max=5000),
         Ch.Params(average_bits=14, seed=0, min=9000, max=70000)][case % 3]
    n = int(rng.integers(1, 60))
    lens = rng.integers(0, 4 * p.max, n)
    lens[rng.random(n) < 0.15] = 0
    batch_bytes = int(rng.choice([1 << 30, 3 * p.max, 50_000]))
    lines, data = run(consumer, tmp_path, p, batch_bytes, lens)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)

    # 1. the batch scan with Ref ids
    segs, _ = coracle.segment_files(data, offs, p, nthreads=4)
    got = [ln.split()[1:] for ln in lines if ln.startswith("seg ")]
    assert len(got) == len(segs)
    for g, s in zip(got, segs):
        assert [int(x) for x in g[:4]] == [int(s["file"]), int(s["offset"]), int(s["size"]),
                                          int(s["flags"])]
        assert g[4] == bytes(s["hash"]).hex()
        a = int(offs[s["file"]] + s["offset"])
        rid, dek = Ch.create_ref_id(data[a:a + int(s["size"])].tobytes())
        assert (g[5], g[6]) == (rid.hex(), dek.hex())

    # 2. the chunk.Writer mirror: every callback, in order
    files = [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in range(n)]
    chunks = Ch.chunk_stream(files, p, segmenter="numpy", with_ref_id=True)
    want = []
    for ch in chunks:
        want.append("cb %d" % len(ch.annotations))
        for a in ch.annotations:
            d = a.next_data_ref
            want.append("ann %d 0" % a.data if d is None else
                        "ann %d 1 %d %d %d %s %s %s %d %d" % (
                            a.data, ch.index, len(ch.data), int(ch.edge), d.ref.id.hex(),
                            d.ref.dek.hex(), d.hash.hex(), d.offset_bytes, d.size_bytes))
    want.append("counts %d %d" % (len(chunks), n))
    assert [ln for ln in lines if not ln.startswith("seg ")] == want


@pytest.fixture(scope="module")
def group_consumer(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("c") / "group_consumer")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "group_consumer.c"),
                    "-L", libdir, "-lpfscdc", "-Wl,-rpath," + libdir,
                    "-Wl,-rpath-link,/opt/rocm/lib", "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("ndev", [2, 4, 8])
def test_c_process_drives_a_device_group(group_consumer, tmp_path, ndev):
    """A plain C process creates a device group of ndev contexts (all on the one GPU here),
    scans a batch over it and runs an unordered writer over it: the program itself checks
    both against one ctx byte for byte (records, Refs, per-file ranges; the ordered event
    stream and every fileset root); here its dealing is checked against pfscdc_deal and its
    records against the oracle."""
    from pfs_amd.group import deal

    rng = np.random.default_rng(6100 + ndev)
    p = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
    n = 300
    lens = rng.integers(0, 3 * p.max, n)
    lens[rng.random(n) < 0.1] = 0
    data_path = str(tmp_path / "data.bin")
    res = subprocess.run([group_consumer, data_path, str(ndev), str(p.average_bits), str(p.seed),
                          str(p.min), str(p.max), "400000", "900000"] +
                         [str(int(x)) for x in lens], capture_output=True, text=True, timeout=100)
    assert res.returncode == 0, res.stderr
    lines = res.stdout.splitlines()
    data = np.fromfile(data_path, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    pb = deal(offs, ndev)
    assert [ln for ln in lines if ln.startswith("part ")] == \
        ["part %d %d %d" % (k, pb[k], pb[k + 1]) for k in range(ndev)]
    segs, _ = coracle.segment_files(data, offs, p, nthreads=4)
    got = [ln.split()[1:] for ln in lines if ln.startswith("seg ")]
    assert len(got) == len(segs)
    for g, s in zip(got, segs):
        assert [int(x) for x in g[:4]] == [int(s["file"]), int(s["offset"]), int(s["size"]),
                                          int(s["flags"])]
        assert g[4] == bytes(s["hash"]).hex()
    assert len([ln for ln in lines if ln.startswith("stream ")]) == 1
    uw = [ln.split() for ln in lines if ln.startswith("uw ")]
    assert len(uw) == 1 and int(uw[0][1]) > 0 and int(uw[0][2]) >= 2 * ndev
