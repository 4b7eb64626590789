"""Static audit of the DPP wait states in the product kernels (CPU only: hipcc cross-compiles).

The broadcast-FMA asm blocks (csrc/pdipm_srbd.hpp SRBD_FMAC_BC) open with `s_nop 1` and carry no
trailing wait states; the compiler pads its own DPPs after a block. A wrong wait state gives wrong
values with no fault, and possibly only under some wave interleavings, so the final ISA of both
translation units is checked: no DPP instruction reads a VGPR written within the 2 wait states before
it (scripts/dpp_hazard_check.py; a planted hazard is detected by the same checker).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CSRC = os.path.join(ROOT, "biped_pympc_amd", "csrc")


def _isa(tmp_path, unit, flags):
    out = tmp_path / (unit + ".s")
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", os.path.join(ROOT, "include"),
           "--cuda-device-only", "-S", "-o", str(out), os.path.join(CSRC, unit)] + flags
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return str(out)


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="hipcc not available")
@pytest.mark.parametrize("unit,flags", [
    ("srbd_mpc.hip", ["-DSRBD_SPLIT_REG20"]),  # the main unit as biped_pympc_amd/build.py builds it
    ("srbd_reg20.hip", ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"]),
])
def test_no_dpp_read_within_two_states_of_a_write(tmp_path, unit, flags):
    from dpp_hazard_check import check
    assert check(_isa(tmp_path, unit, flags)) == 0


def test_checker_detects_a_planted_hazard(tmp_path):
    from dpp_hazard_check import check
    p = tmp_path / "t.s"
    p.write_text("_Zk:\n\tv_add_f64 v[2:3], v[4:5], v[6:7]\n\ts_nop 0\n"
                 "\tv_mov_b64_dpp v[8:9], v[2:3] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_endpgm\n")
    assert check(str(p)) == 1
