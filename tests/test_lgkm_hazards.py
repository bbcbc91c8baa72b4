"""The scan kernels issue their table lookups as inline-asm ds_read with hand-counted
s_waitcnt lgkmcnt (cdc_kernels.hip PFS_ROLL64G and the wide form).  The compiler takes an asm
output as ready at once, so it may reuse, copy or spill an in-flight destination register
before the wait: the first build of the (since removed) pair form reused the unused fourth word of a ds_read_b128
destination as a temporary, and its cuts changed from run to run on 128 GiB while the small
parity cases passed.  This compiles the device code and checks that no instruction touches an
LDS read's destination before a wait retires it (tools/lgkm_hazard_check.py).  CPU only."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
CHECK = os.path.join(ROOT, "tools/lgkm_hazard_check.py")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_no_use_of_an_lds_read_before_its_wait(tmp_path):
    out = tmp_path / "dev.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip",
                    "--cuda-device-only", "-S", os.path.join(ROOT, "pfs_amd/csrc/cdc_kernels.hip"),
                    "-o", str(out)], check=True, capture_output=True, cwd=str(tmp_path))
    r = subprocess.run([sys.executable, CHECK, str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:]
    assert r.stdout.count("cdc_scan_kernel") == 2  # the two scan forms were checked


def _check(tmp_path, body):
    f = tmp_path / "snippet.s"
    f.write_text("k:\n" + body + "  s_endpgm\n")
    r = subprocess.run([sys.executable, CHECK, str(f)], capture_output=True, text=True)
    return r.returncode, r.stdout


def test_checker_reports_planted_hazards(tmp_path):
    # a temporary written into an in-flight destination (the pair-form bug)
    rc, out = _check(tmp_path, "  ds_read_b128 v[8:11], v0\n  v_mov_b32 v9, v1\n"
                               "  s_waitcnt lgkmcnt(0)\n")
    assert rc == 1 and "1 hazard" in out, out
    # a copy of a destination before its wait
    rc, out = _check(tmp_path, "  ds_read_b64 v[2:3], v0\n  ds_read_b64 v[4:5], v0\n"
                               "  s_waitcnt lgkmcnt(1)\n  v_mov_b32 v6, v4\n")
    assert rc == 1, out
    # counted waits that retire exactly what is used are fine
    rc, out = _check(tmp_path, "  ds_read_b64 v[2:3], v0\n  ds_read_b64 v[4:5], v0\n"
                               "  s_waitcnt lgkmcnt(1)\n  v_mov_b32 v6, v2\n"
                               "  s_waitcnt lgkmcnt(0)\n  v_xor_b32 v7, v4, v5\n")
    assert rc == 0 and "0 hazard" in out, out
    # in a function with asm markers only asm-issued reads are tracked (the compiler's own
    # reads are its waitcnt pass's business; a linear walk misreads out-of-line blocks)
    rc, out = _check(tmp_path, "  ;;#ASMSTART\n  ds_read_b64 v[2:3], v0\n  ;;#ASMEND\n"
                               "  ds_read_b64 v[4:5], v0\n  v_mov_b32 v4, v1\n"
                               "  v_mov_b32 v7, v3\n"
                               "  s_waitcnt lgkmcnt(1)\n  v_mov_b32 v6, v2\n")
    assert rc == 1 and "1 hazard" in out and "v_mov_b32 v7, v3" in out, out
