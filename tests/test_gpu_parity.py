"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle on the same bytes.

Bar: bit-exact — every segment offset/size/cut flag and every BLAKE2b-256 digest equal to
the restated reference chunker (oracle/cdc_oracle.c, itself cross-checked against the
literal Python Writer and hashlib in the CPU suite).
"""
import hashlib

import numpy as np
import pytest

from conftest import fuzz_cases

from oracle import chunker as Ch
from oracle import coracle
from pfs_amd import _lib
from pfs_amd.cdc import ChunkParams, Chunker, synthetic_bytes

pytestmark = pytest.mark.gpu

SMALL = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
DEFAULT = Ch.Params()


def cp(p: Ch.Params) -> ChunkParams:
    return ChunkParams(p.average_bits, p.seed, p.min, p.max)


_CHUNKERS = {}


def chunker_for(p: Ch.Params) -> Chunker:
    if p not in _CHUNKERS:
        _CHUNKERS[p] = Chunker(cp(p), device=0)
    return _CHUNKERS[p]


def assert_same(gpu_res, data, offs, p, nthreads=8):
    segs, begin = coracle.segment_files(data, offs, p, nthreads=nthreads)
    g = gpu_res.segments
    assert np.array_equal(gpu_res.file_begin, begin), "per-file segment counts differ"
    assert len(g) == len(segs)
    for field in ("offset", "size", "file", "flags"):
        bad = np.nonzero(g[field] != segs[field])[0]
        assert len(bad) == 0, f"{field} differs at segments {bad[:5]}: gpu={g[bad[:5]]} cpu={segs[bad[:5]]}"
    bad = np.nonzero((g["hash"] != segs["hash"]).any(axis=1))[0]
    assert len(bad) == 0, f"digests differ at segments {bad[:5]}"


def random_offsets(rng, nfiles, max_len):
    lens = rng.integers(0, max_len, nfiles)
    return np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_small_params_many_files(seed):
    rng = np.random.default_rng(seed)
    offs = random_offsets(rng, 300, 120_000)
    data = synthetic_bytes(offs, seed)
    assert_same(chunker_for(SMALL).scan(data, offs), data, offs, SMALL)


def test_default_params_multi_mib():
    offs = np.array([0, 3 << 20, (3 << 20) + 12345, (3 << 20) + 12345 + (9 << 20) + 7,
                     (13 << 20) + 999_999, (13 << 20) + 2_000_000], dtype=np.uint64)
    data = synthetic_bytes(offs, 11)
    assert_same(chunker_for(DEFAULT).scan(data, offs), data, offs, DEFAULT)


def test_default_params_long_stream_forces_max():
    # 64 MiB single stream: candidates every ~8 MiB and some 20 MB forced cuts
    offs = np.array([0, 64 << 20], dtype=np.uint64)
    data = synthetic_bytes(offs, 0xC1)
    res = chunker_for(DEFAULT).scan(data, offs)
    assert_same(res, data, offs, DEFAULT)
    assert len(res.segments) >= 4


def test_edge_sizes():
    p = SMALL
    lens = [0, 1, 63, 64, 65, 127, 128, 129, 1999, 2000, 2001, 29999, 30000, 30001, 0, 0,
            60000, 60001, 4096, 12345, 0]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 5)
    assert_same(chunker_for(p).scan(data, offs), data, offs, p)


def test_empty_batches():
    c = chunker_for(SMALL)
    r = c.scan(b"", [0])
    assert len(r.segments) == 0
    r = c.scan(b"", [0, 0, 0])
    assert len(r.segments) == 0 and list(r.file_begin) == [0, 0, 0]


def test_dense_candidates_rescan_path():
    # average_bits=4 makes ~1/16 of positions candidates: every tile overflows its 15 slots
    p = Ch.Params(average_bits=4, seed=1, min=100, max=5000)
    rng = np.random.default_rng(9)
    offs = random_offsets(rng, 40, 300_000)
    data = synthetic_bytes(offs, 9)
    assert_same(chunker_for(p).scan(data, offs), data, offs, p)


def test_periodic_data_dense_then_sparse():
    # locally dense tiles (repeating 48-byte pattern) next to random bytes
    p = Ch.Params(average_bits=10, seed=1, min=3000, max=40000)
    pat = np.frombuffer(bytes(range(48)), dtype=np.uint8)
    rnd = synthetic_bytes([0, 3 << 20], 4)
    blocks = []
    for i in range(6):
        blocks.append(np.tile(pat, (1 << 20) // 48 + 1)[: (1 << 20) + 17 * i])
        blocks.append(rnd[i << 19:(i + 1) << 19])
    data = np.concatenate(blocks)
    offs = np.array([0, len(data) // 3, len(data)], dtype=np.uint64)
    assert_same(chunker_for(p).scan(data, offs), data, offs, p)


def test_wide_mask():
    p = Ch.Params(average_bits=33, seed=3, min=1000, max=9000)
    offs = np.array([0, 500_000, 500_001, 900_000], dtype=np.uint64)
    data = synthetic_bytes(offs, 3)
    assert_same(chunker_for(p).scan(data, offs), data, offs, p)


@pytest.mark.parametrize("bits", [1, 2, 9, 16, 31, 32])
def test_narrow_mask_widths(bits):
    # the narrow scan rolls in a frame rotated by 32 - bits: every width from 1 to 32
    p = Ch.Params(average_bits=bits, seed=1, min=100, max=4000)
    offs = np.array([0, 70_000, 70_001, 200_000], dtype=np.uint64)
    data = synthetic_bytes(offs, 40 + bits)
    assert_same(chunker_for(p).scan(data, offs), data, offs, p)


def test_index_writer_seed0_avgbits20():
    # fileset/index/writer.go:60 uses WithRollingHashConfig(20, 0) (then level+1 seeds)
    for seed in (0, 1, 2):
        p = Ch.Params(average_bits=20, seed=seed, min=1_000_000, max=20_000_000)
        offs = np.array([0, 5 << 20, (5 << 20) + 4_000_000], dtype=np.uint64)
        data = synthetic_bytes(offs, 100 + seed)
        assert_same(chunker_for(p).scan(data, offs), data, offs, p)


@pytest.mark.parametrize("bits", [20, 19])
def test_candidate_list_matches_oracle(bits):
    # ~3 (bits 20) or ~6 (bits 19) candidates per 3 MiB tile, found by different waves and
    # appended to the tile record in arrival order: compaction must sort them; every tile
    # stays sparse (<= 15 stored candidates)
    p = Ch.Params(average_bits=bits, seed=1, min=2000, max=30000)
    n = (9 << 20) + 77
    data = synthetic_bytes([0, n], 21)
    c = chunker_for(p)
    c.scan(data, [0, n])
    gpu = c.debug_candidates()
    assert not np.any(gpu >> np.uint64(63)), "unexpected dense tile"
    cpu = coracle.candidates(data, p)
    assert np.array_equal(gpu, cpu)


def test_device_resident_input_matches_host_input():
    import torch

    p = DEFAULT
    offs = np.array([0] + [(i + 1) * (4 << 20) for i in range(16)], dtype=np.uint64)
    c = chunker_for(p)
    dev = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
    c.fill_synthetic(dev, offs, 0xC2)
    host = synthetic_bytes(offs, 0xC2)
    assert np.array_equal(dev.cpu().numpy(), host), "device synthetic generator differs"
    r_dev = c.scan(dev, offs)
    assert_same(r_dev, host, offs, p)


def test_unaligned_device_pointer_rejected():
    import torch

    c = chunker_for(SMALL)
    dev = torch.zeros(1000, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(_lib.PfsCdcError):
        c.scan(dev[1:], [0, 999])


def test_digests_are_blake2b_of_segment_bytes():
    p = SMALL
    offs = np.array([0, 70_000, 70_000 + 33_333], dtype=np.uint64)
    data = synthetic_bytes(offs, 2)
    r = chunker_for(p).scan(data, offs)
    for s in r.segments:
        a = int(offs[s["file"]] + s["offset"])
        want = hashlib.blake2b(data[a:a + int(s["size"])].tobytes(), digest_size=32).digest()
        assert bytes(s["hash"]) == want


def test_hash_chain_ends_around_the_quiet_thresholds():
    """The hash kernel runs blocks of a wave's quiet stretch in a separate straight-line loop
    (pairs of blocks while every active quad is >= 5 blocks from its chain's end) and the
    general step otherwise.  Chains whose ends fall 0..40 blocks apart, in waves of 16 quads,
    with partial last blocks, cross every threshold; one quad per wave left alone at the end
    covers the masked fetch for idle quads.  Digests against hashlib (BLAKE2b-256)."""
    rng = np.random.default_rng(77)
    sizes = []
    for base in (1, 4, 5, 6, 9, 64, 300):
        for k in range(48):
            sizes.append(128 * (base + k % 41) + int(rng.integers(0, 128)))
    sizes += [128 * 2000 + 5]  # a long lone chain after the others end
    sizes = np.array(sizes, dtype=np.uint64)
    begins = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    data = synthetic_bytes(offs, 0x51)
    ch = Chunker(ChunkParams(), 0)
    got = ch.hash_ranges(data, begins, sizes)
    for i in range(len(sizes)):
        a, n = int(begins[i]), int(sizes[i])
        want = hashlib.blake2b(data[a:a + n].tobytes(), digest_size=32).digest()
        assert bytes(got[i]) == want, f"range {i} ({n} B)"


@pytest.mark.parametrize("bits,min_", [(4, 100), (6, 40_000), (10, 262_143), (12, 270_337)])
def test_scan_skips_first_min_bytes_of_each_file(bits, min_):
    """The scan skips the strip steps of a work unit below its first eligible position
    (file start + min - 1: writer.go:167-170 never cuts earlier, the count resets at each
    Annotate).  File lengths around min, around the 8 KiB step and the 256 KiB unit, empty
    files, and a unit crowded with more than 64 small files (scanned whole); dense candidate
    rates make hits fall right at and around every file's first eligible position."""
    p = Ch.Params(average_bits=bits, seed=1, min=min_, max=max(4 * min_, 5000))
    lens = [0, 1, min_ - 1, min_, min_ + 1, 0, 8191, 8192, 8193, 262_144, 262_145,
            3 * 262_144 + 7, min_ + 8192, min_ + 8191, 2 * min_ + 262_144 + 5]
    lens += [700] * 300                       # > 64 files inside one 256 KiB unit
    lens += [1 << 20, (1 << 20) + 4096 * 3, 5 * min_ + 77, 0]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 1000 + bits)
    c = chunker_for(p)
    res = c.scan(data, offs)
    assert_same(res, data, offs, p)
    scanned = c.last_scan_bytes()
    assert 0 < scanned <= int(offs[-1])
    if min_ > 64 * 1024:
        assert scanned < int(offs[-1]), "nothing skipped"


def test_scan_skip_c2_layout_rolls_three_quarters(knob):
    # configs[1]: 4 MiB files, min 1,000,000: the first 999,999 bytes of each file hold no
    # eligible position, 23.8% of the bytes are never rolled (whole 8 KiB steps).  The
    # skipping past settled cuts is off here (it depends on timing); with it on, at most these
    # bytes are rolled
    p = DEFAULT
    offs = np.array([i * (4 << 20) for i in range(9)], dtype=np.uint64)
    data = synthetic_bytes(offs, 0xC2)
    c = chunker_for(p)
    per_file = (4 << 20) - (999_999 // 8192) * 8192
    knob("PFSCDC_SCAN_CUTSKIP", 0)
    assert_same(c.scan(data, offs), data, offs, p)
    assert c.last_scan_bytes() == 8 * per_file
    assert c.last_scan_mode() == _lib.SCAN_SKIPPED_FIRST_MIN
    knob("PFSCDC_SCAN_CUTSKIP", None)
    assert_same(c.scan(data, offs), data, offs, p)
    assert 0 < c.last_scan_bytes() <= 8 * per_file
    assert c.last_scan_mode() == _lib.SCAN_SKIPPED_FIRST_MIN | _lib.SCAN_SKIPPED_CUTS
    knob("PFSCDC_SCAN_SKIP", 0)
    assert_same(c.scan(data, offs), data, offs, p)
    assert c.last_scan_bytes() == int(offs[-1]) and c.last_scan_mode() == 0


def _cut_skip_layout(min_):
    """File lengths around min, the 256 KiB unit and the 8 KiB step, files with several cuts,
    a constant-byte file, empty files, and whole units crowded with more than 64 sub-min
    files between long files (such a unit must take no dispatch slot)."""
    U = 262_144
    lens = [0, 1, min_ - 1, min_, min_ + 1, U - 1, U, U + 1, 2 * min_, 2 * min_ + 8191,
            3 * min_ + U + 5, 0, 5 << 20, (2 << 20) + 77, 9 * min_ + 3, 1 << 20]
    lens += [(2 << 20) + 4096 * k for k in range(40)]
    lens += [700] * 1200 + [(3 << 20) + 11] + [0, 300] * 400 + [4 * min_ + 9]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    return lens, offs


@pytest.mark.parametrize("grid", ["1", "3", ""])
@pytest.mark.parametrize("bits,min_,max_", [(16, 300_000, 1_200_000), (18, 262_145, 700_000),
                                            (17, 400_000, 4_000_000), (23, 300_000, 1_200_000)])
def test_scan_skips_past_settled_first_cuts(knob, grid, bits, min_, max_):
    """The scan takes its units in rank order and a unit whose file's first cut is settled
    skips the strip steps below cut + min (writer.go:167-170 after the reset at the cut).
    Candidates every 2^bits bytes put first cuts right after min; at 2^23 most first cuts
    are forced at max instead; a constant-byte file has a candidate at every position or at
    none (the parity of T[b]).  With one or three scan workgroups the
    earlier ranks have finished when the later ones start, so skipping happens; the full grid
    runs everything at once.  Results must equal the oracle's either way."""
    if grid:
        knob("PFSCDC_SCAN_GRID", grid)
    p = Ch.Params(average_bits=bits, seed=1, min=min_, max=max_)
    lens, offs = _cut_skip_layout(min_)
    data = synthetic_bytes(offs, 300 + bits)
    a, b = int(offs[14]), int(offs[15])  # the 9 * min + 3 file: constant bytes
    data[a:b] = 0x5A
    c = chunker_for(p)
    res = c.scan(data, offs)
    assert_same(res, data, offs, p)
    knob("PFSCDC_SCAN_CUTSKIP", 0)
    c.scan(data, offs)
    static = c.last_scan_bytes()
    knob("PFSCDC_SCAN_CUTSKIP", None)
    c.scan(data, offs)
    rolled = c.last_scan_bytes()
    assert 0 < rolled <= static
    if grid == "1":
        assert rolled < static, "no unit skipped past a settled cut"


def test_scan_cut_skip_off_below_one_unit():
    """min - 1 below one work unit (256 KiB): a unit's eligible positions can belong to two
    files, so the scan keeps the plain form (same results)."""
    p = Ch.Params(average_bits=14, seed=1, min=200_000, max=900_000)
    lens, offs = _cut_skip_layout(200_000)
    data = synthetic_bytes(offs, 77)
    assert_same(chunker_for(p).scan(data, offs), data, offs, p)


def test_kernel_spans_and_clocks_are_recorded():
    """The execution spans and the shader clock of the scan and hash kernels (s_memtime /
    s_memrealtime per wave, pfscdc_last_kernel_clocks) come back with every scan: spans
    positive and within the HIP-event intervals, clocks within the chip's range."""
    import torch

    offs = np.arange(0, 65, dtype=np.uint64) * np.uint64(4 << 20)
    t = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda:0")
    c = Chunker(cp(DEFAULT), 0)
    c.fill_synthetic(t, offs, 3)
    res = c.scan(t, offs)
    assert len(res.segments) >= 64
    tm = c.timings()
    assert 0 < tm["scan_span"] <= tm["scan"] + 0.05 and 0 < tm["hash_span"] <= tm["hash"] + 0.05
    for k in ("scan_mhz", "hash_mhz"):
        assert 400 < tm[k] < 3000, (k, tm[k])
    c.close()


@pytest.mark.parametrize("waves", ["1", "2", "2s"])
@pytest.mark.parametrize("bin_bytes", ["0", "60000", "1000000000000"])
@pytest.mark.parametrize("ref_ids", [False, True])
def test_hash_bins_equal_oracle(bin_bytes, ref_ids, waves, knob):
    """Hash bins (a quad hashes every segment of a file of at most bin_bytes back to back,
    lpt_order_block): digests, and with PFSCDC_OPT_REF_IDS the per-segment Ref.Ids, equal to
    the oracle whether no file, some files or every file forms a bin (empty files and files
    cut into many segments included); at two waves per SIMD the hash launch also runs the
    fair-share issue priority (its launch-wide counter and the capped quiet countdown); "2s":
    the fair share updated every 16 blocks (the PFSCDC_HASH_FAIR_EVERY knob)."""
    knob("PFSCDC_HASH_BIN_BYTES", bin_bytes)
    knob("PFSCDC_HASH_WAVES", waves[0])
    if waves == "2s":
        knob("PFSCDC_HASH_FAIR_EVERY", 16)
    rng = np.random.default_rng(5)
    lens = np.concatenate([rng.integers(0, 70_000, 200), [0, 0, 1, 30_000, 250_000, 0]])
    rng.shuffle(lens)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 23)
    c = Chunker(cp(SMALL), device=0, ref_ids=ref_ids)
    res = c.scan(data, offs)
    assert_same(res, data, offs, SMALL)
    if ref_ids:  # every segment (a sample once hid deks missing past the queue's length:
        refs = res.refs  # a fresh ctx can get the device memory of a previous correct run)
        for i in range(len(res.segments)):
            g = res.segments[i]
            a = int(offs[g["file"]] + g["offset"])
            rid, dek = Ch.create_ref_id(data[a:a + int(g["size"])].tobytes())
            assert bytes(refs[i]["dek"]) == dek and bytes(refs[i]["id"]) == rid, i
    c.close()


def test_scan_edge_layouts_equal_oracle():
    """The narrow scan at every mask width, edge sizes, dense tiles, periodic data and the
    reference parameters."""
    for bits in (1, 4, 9, 20, 23, 31, 32):
        p = Ch.Params(average_bits=bits, seed=bits % 3, min=100, max=4000)
        offs = np.array([0, 70_000, 70_001, 200_000, 263_000], dtype=np.uint64)
        data = synthetic_bytes(offs, 60 + bits)
        assert_same(chunker_for(p).scan(data, offs), data, offs, p)
    lens = [0, 1, 63, 64, 65, 127, 128, 129, 1999, 2000, 2001, 29999, 30000, 30001, 0, 60001]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 6)
    assert_same(chunker_for(SMALL).scan(data, offs), data, offs, SMALL)
    p = Ch.Params(average_bits=10, seed=1, min=3000, max=40000)
    pat = np.frombuffer(bytes(range(48)), dtype=np.uint8)
    data = np.concatenate([np.tile(pat, 30_000), synthetic_bytes([0, 1 << 20], 8)])
    offs = np.array([0, len(data) // 3, len(data)], dtype=np.uint64)
    assert_same(chunker_for(p).scan(data, offs), data, offs, p)
    offs = np.array([0, 3 << 20, (3 << 20) + 12345, (12 << 20) + 7, 22 << 20], dtype=np.uint64)
    data = synthetic_bytes(offs, 12)
    assert_same(chunker_for(DEFAULT).scan(data, offs), data, offs, DEFAULT)


def _fuzz_layout(rng, min_, total_cap):
    """Random batch: runs of empty, tiny (crowding a unit), sub-min, around-min, unit-sized and
    multi-MB files in random order, up to total_cap bytes."""
    U = 262_144
    kinds = [lambda: 0, lambda: int(rng.integers(1, 2_000)), lambda: int(rng.integers(1, min_)),
             lambda: int(min_ + rng.integers(-3, 4)), lambda: int(U + rng.integers(-70, 70)),
             lambda: int(rng.integers(min_, 6 * min_)), lambda: int(rng.integers(2 << 20, 9 << 20))]
    lens, total = [], 0
    while total < total_cap:
        k = int(rng.integers(0, len(kinds)))
        run = int(rng.integers(1, 200 if k <= 1 else 6))
        for _ in range(run):
            n = max(0, kinds[k]())
            lens.append(n)
            total += n
    return np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)


@pytest.mark.parametrize("case", fuzz_cases(16))
def test_cut_skip_random_layouts_equal_oracle(knob, case):
    """Randomised layouts and parameters where the cut-skipping plan is in force (min - 1 at
    least one 256 KiB unit): mixed runs of empty, tiny, sub-min, around-min, unit-sized and
    long files, some files holding constant runs (candidates everywhere or nowhere), on one,
    three or all scan workgroups.  Cuts and digests must equal the oracle's."""
    rng = np.random.default_rng(9000 + case)
    min_ = int(rng.integers(262_145, 1_500_000))
    max_ = int(min_ * rng.uniform(1.2, 6.0))
    bits = int(rng.choice([13, 15, 17, 19, 20, 23]))
    grid = ["1", "3", ""][case % 3]
    if grid:
        knob("PFSCDC_SCAN_GRID", grid)
    p = Ch.Params(average_bits=bits, seed=int(rng.integers(0, 3)), min=min_, max=max_)
    offs = _fuzz_layout(rng, min_, 40 << 20)
    data = synthetic_bytes(offs, 500 + case)
    for f in rng.choice(len(offs) - 1, size=min(6, len(offs) - 1), replace=False):
        a, b = int(offs[f]), int(offs[f + 1])
        if b - a > 1000:
            s = int(rng.integers(a, b - 500))
            data[s:s + int(rng.integers(500, min(b - s, 3 << 20) + 1))] = int(rng.integers(0, 256))
    c = chunker_for(p)
    assert_same(c.scan(data, offs), data, offs, p)
    assert c.last_scan_mode() & _lib.SCAN_SKIPPED_FIRST_MIN


@pytest.mark.parametrize("case", fuzz_cases(4))
def test_reference_params_random_batches_equal_oracle(case):
    """The reference's parameters (avgBits 23, min 1,000,000, max 20,000,000) on random
    batches of ~100-200 MB: file lengths around min and max and the 256 KiB unit, tiny files,
    multi-max files, constant runs that force cuts at max or make every position a
    candidate; cuts and digests equal the oracle's, with the cut-skipping plan in force."""
    rng = np.random.default_rng(8800 + case)
    kinds = [0, 1, 999_999, 1_000_000, 1_000_001, 262_144, 19_999_999, 20_000_000, 20_000_001,
             4 << 20, 10_737_418]
    lens, total = [], 0
    while total < int(rng.integers(100, 200)) << 20:
        k = rng.random()
        if k < 0.2:  # a run of tiny files (crowding a scan unit)
            run = [int(x) for x in rng.integers(0, 3000, int(rng.integers(1, 150)))]
            lens += run
            total += sum(run)
            continue
        n = int(rng.choice(kinds)) if k < 0.6 else int(rng.integers(0, 25_000_000))
        lens.append(n)
        total += n
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 900 + case)
    for _ in range(int(rng.integers(1, 4))):
        a = int(rng.integers(0, total))
        data[a:a + int(rng.integers(1, 30_000_000))] = int(rng.integers(0, 256))
    c = chunker_for(DEFAULT)
    assert_same(c.scan(data, offs), data, offs, DEFAULT)


@pytest.mark.parametrize("case", fuzz_cases(8))
def test_knobs_never_change_results(knob, case):
    """no knob changes a result.  Random layouts and parameters under random
    settings of every scan and hash knob at once (workgroup cap, both skips, hash bins, waves
    per SIMD, fair share and its period), device-resident or host input."""
    import torch

    rng = np.random.default_rng(12000 + case)
    bits = int(rng.integers(12, 24))
    mn = int(rng.choice([2000, 70_000, 262_145, 1_000_000]))
    p = Ch.Params(average_bits=bits, seed=int(rng.integers(0, 3)), min=mn,
                  max=mn + int(rng.integers(1, 4 * (1 << bits) + 2)))
    knob("PFSCDC_SCAN_GRID", int(rng.choice([0, 1, 3, 64])))
    knob("PFSCDC_SCAN_SKIP", int(rng.integers(0, 2)))
    knob("PFSCDC_SCAN_CUTSKIP", int(rng.integers(0, 2)))
    knob("PFSCDC_HASH_BIN_BYTES", int(rng.choice([-1, 0, 60_000, 1 << 40])))
    knob("PFSCDC_HASH_WAVES", int(rng.integers(0, 3)))
    knob("PFSCDC_HASH_FAIR", int(rng.integers(0, 2)))
    knob("PFSCDC_HASH_FAIR_EVERY", int(rng.choice([8, 16, 256, 4096])))
    lens, total = [], 0
    for _ in range(int(rng.integers(1, 120))):
        n = int(rng.integers(0, min(3 * p.max, 8 << 20))) if rng.random() < 0.7 else \
            int(rng.integers(0, 3000))
        if total + n > 150 << 20:
            break
        lens.append(n)
        total += n
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    data = synthetic_bytes(offs, 1200 + case)
    c = Chunker(cp(p), device=0)
    src = torch.from_numpy(data).cuda() if rng.random() < 0.5 else data
    assert_same(c.scan(src, offs), data, offs, p)
    c.close()


def test_invalid_arguments_are_refused_and_the_ctx_stays_usable():
    """Bad offsets (not starting at 0, not ending at the byte count, decreasing), refs that do
    not match the chunks, and unaligned device bytes are refused with an error before any
    kernel runs; the same ctx then scans a valid batch correctly."""
    import torch

    offs = np.array([0, 5000, 90_000, 200_000], dtype=np.uint64)
    data = synthetic_bytes(offs, 77)
    c = Chunker(cp(SMALL), device=0)
    bad = [[1, 5000, 90_000, 200_000], [0, 5000, 90_000, 199_999], [0, 5000, 90_000, 200_001],
           [0, 90_000, 5000, 200_000], [200_000, 0]]
    for b in bad:
        with pytest.raises(_lib.PfsCdcError):
            c.scan(data, b)
        assert_same(c.scan(data, offs), data, offs, SMALL)
    dev = torch.from_numpy(np.concatenate([np.zeros(1, np.uint8), data])).cuda()
    with pytest.raises(_lib.PfsCdcError, match="aligned"):
        c.scan(dev[1:], offs)
    refs = np.zeros(3, dtype=_lib.ref_dtype())
    for b in ([0, 10, 20, 200_001], [0, 20, 10, 200_000]):
        with pytest.raises(_lib.PfsCdcError):
            c.get_chunks(data, b, refs)
    assert_same(c.scan(data, offs), data, offs, SMALL)
    c.close()


@pytest.mark.parametrize("case", fuzz_cases(1))
def test_contexts_in_concurrent_threads_equal_oracle(case):
    """A Go host runs many writers at once, each on its own context; here four threads each
    own a Chunker (ctypes releases the GIL, so the library's calls run concurrently) and scan
    random batches with different parameters, device-resident or host input.  Every result
    equals the oracle's."""
    import threading

    import torch

    params = [SMALL, Ch.Params(average_bits=14, seed=2, min=300_000, max=900_000),
              Ch.Params(average_bits=9, seed=0, min=64, max=5000), DEFAULT]
    errors = []

    def worker(t):
        try:
            rng = np.random.default_rng(777 + 10 * case + t)
            p = params[t]
            c = Chunker(cp(p), device=0)
            for k in range(6):
                lens = [int(x) for x in rng.integers(0, 3 * p.max, int(rng.integers(1, 40)))]
                offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
                data = synthetic_bytes(offs, 100_000 * case + 1000 * t + k)
                src = torch.from_numpy(data).cuda() if k % 2 else data
                res = c.scan(src, offs)
                segs, begin = coracle.segment_files(data, offs, p, nthreads=2)
                assert np.array_equal(res.file_begin, begin), (t, k)
                for f in ("offset", "size", "file", "flags", "hash"):
                    assert np.array_equal(res.segments[f], segs[f]), (t, k, f)
            c.close()
        except Exception as e:  # reported on the main thread
            errors.append((t, repr(e)))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=300)
    assert not any(th.is_alive() for th in threads), "a scan thread hung"
    assert not errors, errors
