"""The device group's dealing (pfscdc_deal, include/pfscdc.h) on the CPU: the C ABI's split
equals the Python harness's shard_files (one process per GPU) on the same sizes, and has the
properties the group relies on: whole items in order, every item dealt once, parts balanced
by bytes to within one item.  No GPU needed (pfscdc_deal is host code)."""
import numpy as np
import pytest

from pfs_amd.distributed import commit_layout, shard_files, shard_filesets
from pfs_amd.group import deal


@pytest.mark.parametrize("case", range(40))
def test_deal_equals_shard_files_and_balances(case):
    rng = np.random.default_rng(case)
    n = int(rng.integers(0, 300))
    sizes = rng.integers(0, [10, 1 << 20, 1 << 40][case % 3], n)
    sizes[rng.random(n) < 0.2] = 0
    parts = int(rng.integers(1, 12))
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    pb = deal(offs, parts)
    assert pb[0] == 0 and pb[-1] == n and np.all(np.diff(pb.astype(np.int64)) >= 0)
    assert [(int(pb[r]), int(pb[r + 1])) for r in range(parts)] == shard_files(sizes, parts)
    total, biggest = int(offs[-1]), int(sizes.max()) if n else 0
    for r in range(parts):
        got = int(offs[pb[r + 1]] - offs[pb[r]])
        assert got <= -(-total // parts) + biggest


def test_deal_edges():
    assert list(deal([0], 4)) == [0, 0, 0, 0, 0]  # no items
    assert list(deal([0, 10], 3)) == [0, 1, 1, 1]  # one item: the first part takes it
    assert list(deal([0, 5, 10, 15, 20], 4)) == [0, 1, 2, 3, 4]
    assert list(deal([0, 0, 0, 0], 2)) == [0, 0, 3]  # empty items: all in the last part
    big = np.array([0, 1 << 62, (1 << 63) + 5], dtype=np.uint64)  # no overflow near 2^64
    assert list(deal(big, 2)) == [0, 2, 2]  # ceil(total / 2) is past the first item
    from pfs_amd import _lib
    with pytest.raises(_lib.PfsCdcError):
        deal([0, 5, 3], 2)  # offsets must be nondecreasing
    with pytest.raises(_lib.PfsCdcError):
        deal([0, 5], 0)


def test_deal_of_a_commit_filesets():
    """configs[3]: 10,000 files of 100 GiB serialized at 1e9 bytes, filesets dealt over 8."""
    sizes = [10_737_418] * 9999 + [10_737_418 + 2400]
    lay = commit_layout(sizes, 10 ** 9)
    fb = lay.fileset_bytes()
    offs = np.concatenate([[0], np.cumsum(fb)]).astype(np.uint64)
    pb = deal(offs, 8)
    assert [(int(pb[r]), int(pb[r + 1])) for r in range(8)] == shard_filesets(lay, 8)
    per = [int(offs[pb[r + 1]] - offs[pb[r]]) for r in range(8)]
    assert max(per) - min(per) <= 10 ** 9
