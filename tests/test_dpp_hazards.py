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
