"""Diagnostic: per-phase cycle breakdown of the fast PDIPM kernel (s_memtime stamps).

Builds a SEPARATE instrumented library (scripts/phase_prof.hpp force-included) into /tmp and loads it via SRBD_LIB;
the product library is untouched. Stamps serialise nothing but add a few instructions per phase.
Run on the GPU box: python scripts/phase_profile.py [N] [B] [K]
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.environ.get("PHASE_LIB")  # prebuilt instrumented library (N = 20: scripts/build_variant.py
#   OUT --no-regn --reg20=-include --reg20=scripts/phase_prof.hpp, stamps in the N = 20 unit only)
if not LIB:
    LIB = "/tmp/libsrbd_mpc_prof.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-include", os.path.join(ROOT, "scripts", "phase_prof.hpp"), "-o", LIB,
                    os.path.join(ROOT, "biped_pympc_amd/csrc/srbd_mpc.hip")], check=True)
os.environ["SRBD_LIB"] = LIB

import numpy as np  # noqa: E402
import torch  # noqa: E402

from biped_pympc_amd import _native, solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
L = _native.lib()
L.srbd_debug_phase_cycles.argtypes = [ctypes.c_void_p]
wl = make_workload(B, N, seed=1)
inputs = [torch.from_numpy(a).cuda() for a in wl.inputs]
bufs = solver.MPCSolveBuffers.allocate(N, B)
solver.mpc_solve(inputs, N, K, buffers=bufs)
torch.cuda.synchronize()
acc = (ctypes.c_ulonglong * 32)()
L.srbd_debug_phase_cycles(acc)  # reset
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
solver.mpc_solve(inputs, N, K, buffers=bufs)
e1.record()
torch.cuda.synchronize()
L.srbd_debug_phase_cycles(acc)
names = ["residuals", "factor: parallel (W, Phi_u blocks, S_ii)", "factor: stage chain (Schur + sweep)",
         "solve: parallel parts (x3)", "solve: fwd/bwd chains (x3)", "step lengths / update",
         "refinement residuals (KKT rows 1, 4)"]
tot = sum(acc[k] for k in range(7))
print(f"N={N} B={B} K={K}: step {e0.elapsed_time(e1):.3f} ms; cycles per QP per iteration (wave 0):")
for k, n in enumerate(names):
    print(f"  {n:45s} {acc[k] / B / K:10.0f}  ({100 * acc[k] / tot:5.1f} %)")
print(f"  {'total':45s} {tot / B / K:10.0f}")
extra = {7: "the chain waited for wave 1 (all steps)", 8: "  of which before step 0",
         9: "wave 1: split -> first stage pair published", 10: "wave 1: producer weights set up"}
for k, n in extra.items():
    if acc[k] or acc[16 + k]:
        print(f"  {n:45s} {acc[k] / B / K:10.0f} (wave 0) {acc[16 + k] / B / K:10.0f} (wave 1)")
if any(acc[16 + k] for k in range(7)):  # wave 1 of a two-wave QP (its own phase boundaries)
    tot1 = sum(acc[16 + k] for k in range(7))
    print("wave 1:")
    for k, n in enumerate(names):
        print(f"  {n:45s} {acc[16 + k] / B / K:10.0f}  ({100 * acc[16 + k] / tot1:5.1f} %)")
    print(f"  {'total':45s} {tot1 / B / K:10.0f}")
