"""Static audit of the DPP wait states in the product kernels (CPU only: hipcc cross-compiles).

The broadcast-FMA asm blocks (csrc/dpp_rows.hpp SRBD_FMAC_BC) open with `s_nop 1` and carry no
trailing wait states, and inside a block a DPP reads no VGPR written by either of the 2 instructions
before it. A wrong wait state gives wrong values with no fault, and possibly only under some wave
interleavings, so the final ISA of both translation units -- compiled with the product build's own
flags (biped_pympc_amd/build.py unit_compile_cmd) -- is checked: no DPP instruction reads ANY VGPR
(routed source, other sources, fmac accumulator) written within the 2 wait states before it, along
every control-flow predecessor (scripts/dpp_hazard_check.py; planted hazards are detected by the same
checker). Where hipcc exists the audit must run: it fails rather than skips.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


REGN_PARTS = 6  # csrc/srbd_regN.hip SRBD_REGN_PART: its horizons in six parts, compiled in parallel


def _isa(tmp_path, unit):
    """Device ISA of one translation unit: a list of .s files (srbd_regN.hip: one per horizon part,
    the parts compiled concurrently with the product flags plus -DSRBD_REGN_PART=k)."""
    from biped_pympc_amd.build import HIPCC, unit_compile_cmd
    if not (os.path.exists(HIPCC) or shutil.which("hipcc")):
        pytest.skip("hipcc not available")
    parts = [[f"-DSRBD_REGN_PART={k}"] for k in range(REGN_PARTS)] if unit == "srbd_regN.hip" else [[]]
    outs, procs = [], []
    for k, defs in enumerate(parts):
        out = tmp_path / f"{unit}.{k}.s"
        cmd = unit_compile_cmd(unit, [*defs, "--cuda-device-only", "-S", "-o", str(out)])
        procs.append(subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True))
        outs.append(str(out))
    for p in procs:
        err = p.communicate()[1]
        assert p.returncode == 0, err[-2000:]
    return outs


def _reg_horizon(name):
    import re
    m = re.search(r"reg_kernelILi(\d+)E", name)
    return int(m.group(1)) if m else None


@pytest.mark.parametrize("unit", ["srbd_mpc.hip", "srbd_reg20.hip", "srbd_regN.hip"])
def test_no_dpp_read_within_two_states_of_a_write(tmp_path, unit):
    """Also, on the same ISA: the register kernels keep every VGPR in registers -- the fused step
    kernel (mpc_step_reg_kernel) and the CCS solver kernel (pdipm_srbd_reg_kernel, the CusADi
    drop-in's path) at every register horizon 2..32 (the QPs of N >= 25 run on four waves, whose
    three inequality-row slots per lane at three waves had spilled 6-30 VGPRs). The
    fused kernel has no spill at all; the CCS kernel's only ones are the
    whole-wave save of its SGPR-spill register around the call of the in-launch general fallback
    (pdipm.hpp pdipm_general_scratch), which runs for QPs that are not stage-invariant only: no spill
    or reload instruction elsewhere, and at most 2 such registers. And every register kernel stays
    within 256 VGPRs, its callees included (the kernel's count is the maximum over the call graph: a
    fallback phase compiled past 256 would take the fast path from 2 waves per SIMD to 1)."""
    from dpp_hazard_check import check
    from kernel_resources import body_spills, resources
    seen = set()
    for s in _isa(tmp_path, unit):
        assert check(s) == 0, s
        for name, r in resources(s, "reg_kernel").items():
            n = _reg_horizon(name)
            if n is not None:
                assert r["vgpr_count"] <= 256, (name, r)
                if "mpc_step" in name:
                    assert r["vgpr_spill_count"] == 0, (name, r)
                else:
                    assert r["vgpr_spill_count"] <= 2, (name, r)
                    assert body_spills(s, name) == [], (name, body_spills(s, name))
                seen.add(("mpc_step" in name, n))
    if unit == "srbd_regN.hip":  # every horizon of the unit was audited, both kernels
        assert seen == {(f, n) for f in (False, True) for n in range(2, 33) if n not in (10, 20)}, seen


def test_checker_detects_planted_hazards(tmp_path):
    from dpp_hazard_check import check
    cases = {
        # routed source written 1 state before
        "src0": "_Zk:\n\tv_add_f64 v[2:3], v[4:5], v[6:7]\n\ts_nop 0\n"
                "\tv_mov_b64_dpp v[8:9], v[2:3] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_endpgm\n",
        # fmac accumulator written by the previous instruction
        "acc": "_Zk:\n\tv_fmac_f64_dpp v[2:3], v[4:5], v[6:7] row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
               "\tv_fmac_f64_dpp v[2:3], v[4:5], v[8:9] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\ts_endpgm\n",
        # written before a branch whose target is right in front of the DPP
        "branch": "_Zk:\n\tv_add_f64 v[2:3], v[4:5], v[6:7]\n\ts_branch .LBB0_2\n\ts_nop 7\n.LBB0_2:\n"
                  "\tv_mov_b64_dpp v[8:9], v[2:3] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_endpgm\n",
    }
    for name, text in cases.items():
        p = tmp_path / f"{name}.s"
        p.write_text(text)
        assert check(str(p), verbose=False) == 1, name
    ok = tmp_path / "ok.s"
    ok.write_text("_Zk:\n\tv_add_f64 v[2:3], v[4:5], v[6:7]\n\ts_nop 1\n"
                  "\tv_mov_b64_dpp v[8:9], v[2:3] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\ts_endpgm\n")
    assert check(str(ok), verbose=False) == 0
