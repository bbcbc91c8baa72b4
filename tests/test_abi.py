"""C ABI checks that need no GPU: libpfscdc.so loads, exports every function declared in
include/pfscdc.h, and its host-side pieces (table generation, Go rand) are correct.
No compute calls on the device here."""
import ctypes as C
import os
import re
import subprocess
import sys

import pytest

from oracle import buzhash64, gorand
from pfs_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pfscdc.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(pfscdc_[a-z0-9_]+)\s*\(", text))
    return sorted(n for n in names if not n.endswith("_cb"))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.run(["make", "-s", "-C", ROOT, "pfs_amd/libpfscdc.so"], check=True)
    return _lib.load()


def test_header_and_binding_agree(lib):
    assert declared_functions() == sorted(_lib.EXPORTED)


def test_every_declared_symbol_is_exported(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (pfscdc_\w+)", out))
    assert set(declared_functions()) <= exported


def test_library_is_gfx950_code_object(lib):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list",
                          "--type=o", f"--input={_lib.LIB_PATH}"], capture_output=True, text=True)
    if out.returncode == 0 and out.stdout:
        assert "gfx950" in out.stdout
    else:  # fall back to scanning the fat binary for the target id
        assert b"gfx950" in open(_lib.LIB_PATH, "rb").read()


def test_default_params(lib):
    p = _lib.default_params()
    assert (p.average_bits, p.seed, p.min_chunk, p.max_chunk) == (23, 1, 1_000_000, 20_000_000)


@pytest.mark.parametrize("seed", [0, 1, 2, 3, -7, 1 << 40])
def test_native_table_equals_oracle(lib, seed):
    assert _lib.table(seed) == buzhash64.generate_hashes(seed)


def test_native_go_rand_equals_oracle(lib):
    for seed in (0, 1, 99, -123456789):
        src = gorand.Source(seed)
        assert _lib.go_int63(seed, 20) == [src.int63() for _ in range(20)]


def test_ctx_create_rejects_bad_params(lib):
    ctx = C.c_void_p()
    p = _lib.Params(23, 0, 1, 32, 1000)  # min < 64: unsupported on the GPU path
    assert lib.pfscdc_ctx_create(C.byref(p), 0, C.byref(ctx)) == _lib.PFSCDC_EUNSUPPORTED
    p = _lib.Params(23, 0, 1, 5000, 1000)  # max < min
    assert lib.pfscdc_ctx_create(C.byref(p), 0, C.byref(ctx)) == _lib.PFSCDC_EINVAL


INTEGRATION = os.path.join(ROOT, "INTEGRATION.md")


def documented_knobs():
    """The first column of INTEGRATION.md's knob table: name -> (default, lo, hi)."""
    text = open(INTEGRATION).read()
    table = text.split("<!-- knob list:", 1)[1]
    out = {}
    for m in re.finditer(r"^\| `(PFSCDC_[A-Z0-9_]+)` \| (-?\d+) \| (-?\d+)–(\S+) \|", table, re.M):
        hi = m.group(4)
        hi = 1 << int(hi[2:]) if hi.startswith("2^") else int(hi)
        out[m.group(1)] = (int(m.group(2)), int(m.group(3)), hi)
    return out


def header_macros():
    return set(re.findall(r"#define\s+(PFSCDC_[A-Z0-9_]+)", open(HEADER).read()))


def test_knob_table_equals_integration_list(lib):
    """The knobs the library has are exactly the documented ones, with their defaults and
    ranges (no undocumented A/B branch a stray variable could select)."""
    doc = documented_knobs()
    lib_knobs = _lib.knob_info()
    assert set(lib_knobs) == set(doc)
    for name, (lo, hi, d) in lib_knobs.items():
        assert doc[name] == (d, lo, hi), name


def test_library_strings_name_only_documented_knobs(lib):
    """Every PFSCDC_* string inside libpfscdc.so (what a getenv could name) is a documented
    knob or a macro of the public header (option names in error messages)."""
    blob = open(_lib.LIB_PATH, "rb").read()
    found = {m.decode() for m in re.findall(rb"PFSCDC_[A-Z0-9_]+", blob)}
    allowed = set(documented_knobs()) | header_macros()
    assert found - allowed == set(), sorted(found - allowed)
    assert set(documented_knobs()) <= found


def test_sources_read_the_environment_only_in_knobs_cpp():
    """getenv / environ appear only in knobs.cpp."""
    csrc = os.path.join(ROOT, "pfs_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f == "knobs.cpp" or not f.endswith((".cpp", ".hip", ".h")):
            continue
        for ln, line in enumerate(open(os.path.join(csrc, f)), 1):
            code = line.split("//", 1)[0]
            assert "getenv" not in code and "environ" not in code, \
                f"{f}:{ln} reads the environment outside knobs.cpp"


def test_product_source_has_no_compile_time_experiments():
    """The product library is one build: no A/B macros, no development-only branches
    (VERDICT r5 item 4).  Only the public header's include guard and extern "C" use the
    preprocessor's conditionals."""
    pat = re.compile(r"PFS_EXP_|PFS_SCAN_DYN|PFS_HASH_CXX|PFS_HASH_LANES|PFS_WAVE_TRACE")
    for d in (os.path.join(ROOT, "pfs_amd", "csrc"), os.path.join(ROOT, "include")):
        for f in sorted(os.listdir(d)):
            if not f.endswith((".cpp", ".hip", ".h")):
                continue
            text = open(os.path.join(d, f)).read()
            assert not pat.search(text), f
            conds = [l.strip() for l in text.splitlines() if l.strip().startswith("#if")]
            allowed = {"#ifndef PFSCDC_H", "#ifdef __cplusplus"}
            assert set(conds) <= allowed, (f, conds)


def test_knob_set_get_and_ranges(lib):
    d = _lib.get_knob("PFSCDC_SCAN_GRID")
    with _lib.knobs(PFSCDC_SCAN_GRID=7):
        assert _lib.get_knob("PFSCDC_SCAN_GRID") == 7
    assert _lib.get_knob("PFSCDC_SCAN_GRID") == d
    assert lib.pfscdc_set_knob(b"PFSCDC_HASH_WAVES", 9) == _lib.PFSCDC_EINVAL  # above 8
    assert lib.pfscdc_set_knob(b"PFSCDC_SCAN_PAIR", 1) == _lib.PFSCDC_EINVAL  # removed form
    v = C.c_int64()
    assert lib.pfscdc_get_knob(b"PFSCDC_NOPE", C.byref(v)) == _lib.PFSCDC_EINVAL
    assert lib.pfscdc_knob_info(-1, None, None, None) is None


def test_environment_is_read_once_with_bad_values_ignored(tmp_path):
    """A fresh process: a good variable sets its knob, a bad one keeps the default (and says
    so on stderr), a removed A/B variable is ignored."""
    code = ("from pfs_amd import _lib; import sys; "
            "print(_lib.get_knob('PFSCDC_SCAN_GRID'), _lib.get_knob('PFSCDC_HASH_WAVES'), "
            "_lib.get_knob('PFSCDC_COMMIT_LONG_PCT'))")
    env = dict(os.environ, PFSCDC_SCAN_GRID="64", PFSCDC_HASH_WAVES="x", PFSCDC_COMMIT_LONG_PCT="100",
               PFSCDC_SCAN_PAIR="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, cwd=ROOT,
                       check=True)
    assert r.stdout.split() == ["64", "0", "30"]
    assert "PFSCDC_HASH_WAVES=x" in r.stderr and "PFSCDC_COMMIT_LONG_PCT=100" in r.stderr
    assert "ignoring PFSCDC_SCAN_PAIR (not a knob" in r.stderr  # a retired name is reported
    assert "ignoring PFSCDC_SCAN_GRID" not in r.stderr


def test_product_does_not_import_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "pfs_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", src).replace("\"oracle\"", ""), f


def _header_arities():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for name, params in re.findall(r"\b(pfscdc_[a-z0-9_]+)\s*\(([^()]*)\)\s*;", text):
        p = params.strip()
        out[name] = 0 if p in ("", "void") else p.count(",") + 1
    return out


def _calls(code):
    """(name, argument count) of every pfscdc_* call in code (top-level commas)."""
    for m in re.finditer(r"\b(?:C\.)?(pfscdc_[a-z0-9_]+)\(", code):
        depth, i, args, nonblank = 1, m.end(), 0, False
        while depth:
            ch = code[i]
            if ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
            elif ch == "," and depth == 1:
                args += 1
            if depth and not ch.isspace():
                nonblank = True
            i += 1
        yield m.group(1), (args + 1 if nonblank else 0)


def test_cgo_stub_matches_header():
    """The cgo binding in INTEGRATION.md (the reference-side stub a maintainer would add)
    calls only functions pfscdc.h declares, each with its prototype's argument count, and
    never hands C a Go pointer to keep (the cgo.Handle travels as an integer)."""
    ar = _header_arities()
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```go\n(.*?)```", doc, flags=re.S)
    assert blocks
    seen = set()
    for code in blocks:
        code = re.sub(r"//[^\n]*", "", code)  # comments
        for name, n in _calls(code):
            assert name in ar, name
            assert n == ar[name], (name, n, ar[name])
            seen.add(name)
        assert "unsafe.Pointer(&g.handle)" not in code
    for required in ("pfscdc_ctx_create", "pfscdc_writer_create", "pfscdc_writer_annotate",
                     "pfscdc_writer_write", "pfscdc_writer_close", "pfscdc_set_options",
                     "pfscdc_writer_set_store", "pfscdc_store_get", "pfscdc_writer_copy"):
        assert required in seen, required


def _go_blocks():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return [re.sub(r"//[^\n]*", "", b) for b in re.findall(r"```go\n(.*?)```", doc, flags=re.S)]


# Go APIs newer than the reference's toolchain (go.mod:3 `go 1.16`, etc/compile/GO_VERSION
# 1.16.4), with the release that added them
_GO_AFTER_116 = {
    r'"runtime/cgo"': "1.17", r"\bcgo\.(New)?Handle\b": "1.17", r"\bunsafe\.Slice\b": "1.17",
    r"\bunsafe\.Add\b": "1.17", r"\bunsafe\.(SliceData|String|StringData)\b": "1.20",
    r"\batomic\.(Int32|Int64|Uint32|Uint64|Bool|Pointer|Uintptr)\b": "1.19",
    r"\bany\b": "1.18", r"\[\s*\w+\s+(any|comparable)\s*\]": "1.18",
    r"\bstrings\.Cut\b": "1.18", r"\b(min|max|clear)\(": "1.21", r"\bslices\.|\bmaps\.": "1.21",
}


def test_cgo_stub_is_go116():
    """The stub compiles under Go 1.16: no runtime/cgo.Handle, unsafe.Slice, generics or
    later library APIs."""
    for code in _go_blocks():
        for pat, ver in _GO_AFTER_116.items():
            # parameter names min/max in a signature are identifiers, not the 1.21 builtins
            hits = [m for m in re.finditer(pat, code)
                    if not (pat.startswith(r"\b(min|max") and code[m.start() - 1:m.start()] in ", ")]
            assert not hits, (pat, ver, code[hits[0].start() - 40:hits[0].end() + 40])


def test_cgo_stub_never_rehashes_on_the_host():
    """Uploads go through CreateWithID with the GPU's Ref.Id: no client.Create( call (its
    Hash(chunkData), client.go:57, would re-hash the ciphertext) and no chunk.Hash."""
    code = "\n".join(_go_blocks())
    assert not re.search(r"\bclient\.Create\(|\.Create\(g\.ctx", code)
    assert not re.search(r"(?<![\w.])Hash\(", code)
    assert "CreateWithID(" in code


def _apply_hunk(text, hunk):
    """Apply one unified-diff hunk (context/removals must match exactly) to text."""
    old, new = [], []
    for line in hunk.splitlines():
        if line.startswith(("---", "+++", "@@")):
            continue
        tag, body = (line[:1], line[1:]) if line else (" ", "")
        if tag in " -":
            old.append(body)
        if tag in " +":
            new.append(body)
    old_s, new_s = "\n".join(old) + "\n", "\n".join(new) + "\n"
    assert text.count(old_s) == 1, "hunk context does not match client.go"
    return text.replace(old_s, new_s)


REF_CLIENT = "/root/reference/src/internal/storage/chunk/client.go"


@pytest.mark.skipif(not os.path.exists(REF_CLIENT), reason="reference tree not present")
def test_create_with_id_patch_applies():
    """The one reference-side patch applies to chunk/client.go as it lies in
    the reference, keeps Create's behaviour (Create = CreateWithID(Hash(chunkData))) and
    leaves the hash nowhere else."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    (hunk,) = re.findall(r"```diff\n(.*?)```", doc, flags=re.S)
    assert "a/src/internal/storage/chunk/client.go" in hunk
    out = _apply_hunk(open(REF_CLIENT).read(), hunk)
    assert out.count("Hash(chunkData)") == 1
    create = out[out.index("func (c *trackedClient) Create("):out.index("func (c *trackedClient) CreateWithID(")]
    assert "return c.CreateWithID(ctx, md, Hash(chunkData), chunkData)" in create
    with_id = out[out.index("func (c *trackedClient) CreateWithID("):out.index("func (c *trackedClient) Get(")]
    assert "chunkID :=" not in with_id and "c.store.Put(ctx, key, chunkData)" in with_id


def test_plain_c_consumer_builds_and_agrees_with_oracle(lib, tmp_path):
    """include/pfscdc.h compiles as strict C99 (what cgo's C compiler sees) and a C program
    linked against libpfscdc.so gets, from the host-side entry points, the oracle's table and
    Go Int63 stream, fileset.Clean, the store's put/get/dedup and the knob table."""
    from oracle import fileset as OF
    exe = str(tmp_path / "abi_consumer")
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "abi_consumer.c"),
                    "-L", libdir, "-lpfscdc", "-Wl,-rpath," + libdir,
                    "-Wl,-rpath-link,/opt/rocm/lib", "-o", exe], check=True)
    paths = ["a//b/../c", "/", "", "x/", "./y/./z/..", "dir/sub/"]
    seed = -7
    res = subprocess.run([exe, str(seed)] + paths, capture_output=True, text=True, check=True)
    lines = res.stdout.splitlines()
    fields = {}
    for ln in lines:
        fields.setdefault(ln.split()[0], []).append(ln.split()[1:])
    assert fields["params"] == [["23", "1", "1000000", "20000000"]]
    assert [int(x, 16) for x in fields["table"][0]] == buzhash64.generate_hashes(seed)
    src = gorand.Source(seed)
    assert [int(x) for x in fields["int63"][0]] == [src.int63() for _ in range(8)]
    codes = dict(re.findall(r"#define (PFSCDC_E\w+) (-\d+)", open(HEADER).read()))
    assert fields["store"] == [["count", "1", "missing", codes["PFSCDC_ENOTFOUND"]]]
    assert fields["ctx_null"] == [[codes["PFSCDC_EINVAL"]]]
    assert fields["unknown_knob"] == [[codes["PFSCDC_EINVAL"]]]
    assert [(k[0], tuple(int(x) for x in k[1:])) for k in fields["knob"]] == \
        list(_lib.knob_info().items())
    want = [[str(d), OF.clean(p, bool(d))] for p in paths for d in (0, 1)]
    assert fields["clean"] == want


@pytest.mark.parametrize("name", ["abi_consumer", "abi_gpu_consumer", "uw_consumer"])
def test_c_drivers_build_strict(lib, tmp_path, name):
    """Every C driver of the ABI (tests/c/: the CPU consumer, the GPU consumer, the host-
    sanitizer driver) compiles and links as strict C99 against the header and library."""
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-pedantic", "-Werror",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", name + ".c"),
                    "-L", libdir, "-lpfscdc", "-Wl,-rpath," + libdir,
                    "-Wl,-rpath-link,/opt/rocm/lib", "-o", str(tmp_path / name)], check=True)
