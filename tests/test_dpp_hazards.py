"""The hash kernel's inline-asm rounds read a, c and d through DPP operands with no s_nop in
front (gfx9 needs 2 wait states between a VALU write of a VGPR and a DPP read of it, and the
hardware does not interlock).  That is safe only while the compiler places no VALU write of
those registers right before a round; this test compiles the device code and checks every DPP
instruction of the library (tools/dpp_hazard_check.py).  CPU only: hipcc cross-compiles."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_no_dpp_read_after_valu_write_hazard(tmp_path):
    out = tmp_path / "dev.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-x", "hip",
                    "--cuda-device-only", "-S", os.path.join(ROOT, "pfs_amd/csrc/cdc_kernels.hip"),
                    "-o", str(out)], check=True, capture_output=True, cwd=str(tmp_path))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools/dpp_hazard_check.py"), str(out)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "dpp hazards: 0" in r.stdout


def _check(tmp_path, text):
    f = tmp_path / "snippet.s"
    f.write_text(text)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools/dpp_hazard_check.py"), str(f)],
                       capture_output=True, text=True)
    return r.returncode, r.stdout


@pytest.mark.parametrize("dpp", [
    # VOP1 DPP: the source is the last operand, followed by its modifiers
    "v_mov_b32_dpp v1, v2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
    # VOP2 DPP with the source in the middle
    "v_xor_b32_dpp v1, v2, v5 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf",
    # carry form: dst, vcc, src0
    "v_add_co_u32_dpp v1, vcc, v2, v5 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf",
    "v_mov_b32_dpp v1, v2 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1",
])
def test_checker_reports_a_planted_hazard(tmp_path, dpp):
    """Self-test: the checker must see the DPP source wherever it sits."""
    rc, out = _check(tmp_path, f"k:\n  v_add_u32 v2, v3, v4\n  {dpp}\n  s_endpgm\n")
    assert rc == 1 and "dpp hazards: 1" in out, out
    # two wait states in between make it safe
    rc, out = _check(tmp_path, f"k:\n  v_add_u32 v2, v3, v4\n  s_nop 1\n  {dpp}\n  s_endpgm\n")
    assert rc == 0 and "dpp hazards: 0" in out, out
