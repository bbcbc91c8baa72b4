"""The parity pin one command away: oracle/go_probe/main.go prints the
real buzhash64.GenerateHashes tables and the chunk.Writer.roll segments of the first two golden
cases; expected_int63.txt / expected_uint64.txt are what it prints under each reading of
assumption A1.  Checked here without Go: both files equal a fresh oracle run, the int63 file
is exactly the committed golden vectors (so one `go run` + diff checks those), and the two
variants differ (so the diff decides between them)."""
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "oracle", "go_probe")
sys.path.insert(0, PROBE)
import expected  # noqa: E402


def read(name):
    return open(os.path.join(PROBE, name)).read()


@pytest.mark.parametrize("draw", ["int63", "uint64"])
def test_expected_files_equal_a_fresh_oracle_run(draw):
    assert read("expected_%s.txt" % draw) == expected.render(draw)


def test_lens_go_is_generated():
    assert read("lens.go") == expected.lens_go()


def test_int63_variant_is_the_golden_vectors():
    golden = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    lines = read("expected_int63.txt").splitlines()
    for seed in ("0", "1", "2"):
        t = golden["tables"][seed]
        for i in (0, 1, 2, 3, 255):
            assert "table %s %d %s" % (seed, i, t[i]) in lines
    for case in golden["cases"][:2]:
        k = lines.index("case " + case["name"])
        segs = []
        for ln in lines[k + 1:]:
            if not ln.startswith("seg "):
                break
            f, o, s, cut, h = ln.split()[1:]
            segs.append([int(f), int(o), int(s), int(cut), h])
        assert segs == case["segments"], case["name"]


def test_the_two_variants_are_told_apart():
    a, b = read("expected_int63.txt").splitlines(), read("expected_uint64.txt").splitlines()
    ta = [ln for ln in a if ln.startswith("table ")]
    tb = [ln for ln in b if ln.startswith("table ")]
    assert ta != tb
    assert [ln for ln in a if ln.startswith("seg ")] != [ln for ln in b if ln.startswith("seg ")]


def test_probe_is_go116_and_pins_the_reference_modules():
    src = read("main.go")
    assert "buzhash64.GenerateHashes(" in src and "blake2b.Sum256(" in src
    for pat in (r"\bany\b", r"\[\s*\w+\s+(any|comparable)\s*\]", r"\bunsafe\.", r"\bslices\.",
                r"\bmaps\.", r"\bstrings\.Cut\b"):
        assert not re.search(pat, re.sub(r"//[^\n]*", "", src)), pat
    mod = read("go.mod")
    assert "go 1.16" in mod
    ref = "/root/reference/go.mod"
    if os.path.exists(ref):
        text = open(ref).read()
        for dep in ("github.com/chmduquesne/rollinghash v4.0.0+incompatible",
                    "golang.org/x/crypto v0.0.0-20201208171446-5f87f3452ae9"):
            assert dep in text and dep in mod
