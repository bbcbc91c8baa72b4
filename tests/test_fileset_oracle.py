"""CPU tests of the stream-formation oracle (oracle/fileset.py) and the library's path
cleaning, against properties the reference code implies (fileset/unordered_writer.go,
buffer.go, util.go) and Go path.Clean's documented cases."""
import numpy as np
import pytest

from oracle import chunker as Ch
from oracle import fileset as OF

SMALL = Ch.Params(average_bits=12, seed=1, min=2000, max=30000)
SMALL_INDEX = Ch.Params(average_bits=13, seed=0, min=3000, max=60000)


@pytest.mark.parametrize("p,want", [
    ("", "."), ("abc", "abc"), ("a/c", "a/c"), ("a//c", "a/c"), ("a/c/.", "a/c"),
    ("a/c/b/..", "a/c"), ("/../c", "/c"), ("../../abc", "../../abc"), ("/", "/"),
    ("abc/def/../../..", ".."), ("abc/./../def", "def"), ("a/../../b", "../b"),
    ("//abc", "/abc"), ("abc/", "abc"), ("/abc/def/ghi/../jkl", "/abc/def/jkl"),
])
def test_go_path_clean_cases(p, want):
    assert OF.go_path_clean(p) == want


def test_fileset_clean():
    assert OF.clean("", False) == "/"
    assert OF.clean("a/b/", False) == "/a/b"
    assert OF.clean("a/b", True) == "/a/b/"
    assert OF.clean("/x/../", True) == "/"


def test_library_clean_matches_oracle():
    from pfs_amd import fileset as PF
    rng = np.random.default_rng(4)
    parts = ["a", "b", ".", "..", "", "c.d", "..."]
    for _ in range(300):
        p = "/".join(parts[int(i)] for i in rng.integers(0, len(parts), int(rng.integers(0, 6))))
        if rng.integers(0, 2):
            p = "/" + p
        for d in (False, True):
            assert PF.clean(p, d) == OF.clean(p, d), (p, d)


def test_buffer_sorts_by_path_then_tag_and_keeps_emptied_paths():
    b = OF.Buffer()
    b.add("/b", "t2") .extend(b"1")
    b.add("a", "t9").extend(b"2")
    b.add("/b", "t1").extend(b"3")
    assert [(p, t) for p, t, _ in b.walk_additive()] == [("/a", "t9"), ("/b", "t1"), ("/b", "t2")]
    b.delete("/a", "t9")
    assert not b.empty() and "/a" in b.additive and b.additive["/a"] == {}
    assert b.walk_deletive() == [("/a", "t9")]
    b.delete("/b/", "x")  # directory delete drops buffered files only
    assert "/b" in b.additive  # "/b" does not start with "/b/"


def test_put_splits_at_memory_threshold_and_bytes_are_conserved():
    data = bytes(range(256)) * 1000  # 256,000 B
    uw = OF.UnorderedWriter(SMALL, 100_000, SMALL_INDEX)
    uw.put("/big", "", False, data)
    uw.put("/small", "", False, b"x" * 10)
    fss = uw.close()
    assert [fs.size_bytes for fs in fss] == [100_000, 100_000, 56_010]
    assert [fs.files for fs in fss][0] == [("/big", "default")]
    assert fss[2].files == [("/big", "default"), ("/small", "default")]
    # Put without append deletes first: only the first piece carries the deletive entry
    assert fss[0].deletes == [("/big", "default")] and fss[1].deletes == []


def test_directory_delete_reaches_serialized_filesets():
    uw = OF.UnorderedWriter(SMALL, 50_000, SMALL_INDEX)
    for i in range(6):
        uw.put(f"/d/f{i}", "", True, bytes([i]) * 20_000)
    uw.delete("/d/")
    fss = uw.close()
    # f0..f4 were serialized (f4 fills the second fileset exactly, leaving an empty buffered
    # re-Add of it); the directory delete drops the buffered f4/f5 and deletes f0..f4
    last = fss[-1]
    assert last.files == [] and last.size_bytes == 0
    assert last.deletes == [(f"/d/f{i}", "default") for i in range(5)]


def test_index_root_is_top_level_entry():
    # one file: a single level-0 entry -> level 0 has 1 annotation in 1 chunk -> the root is
    # that entry with its Range set (index/writer.go:143-160)
    uw = OF.UnorderedWriter(SMALL, 10 ** 9, SMALL_INDEX)
    uw.put("/only", "", False, bytes(5000))
    fs = uw.close()[0]
    entries = [e[2] for e in uw.log[0] if e[0] == "index" and e[1] == 0]
    assert len(entries) == 1
    assert fs.additive.startswith(entries[0][8:10])  # same path field first
    assert len(fs.additive) > len(entries[0]) - 8  # plus the Range
