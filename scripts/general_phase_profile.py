"""Diagnostic: per-phase cycles of the general solve (csrc/pdipm.hpp pdipm_general_at) from s_memtime stamps.

  python scripts/general_phase_profile.py build           (build host: instrumented library -> ab/;
                                                           GPROF_LIB=<name> picks the file name)
  python scripts/general_phase_profile.py run [N] [B] [K] (GPU box: general path, prints cycles per QP)

The instrumented library is srbd_mpc.hip compiled with scripts/phase_prof.hpp force-included (the
PROF_* markers become stamps; the product build's are empty), linked with the product's objects of
the other two units. Phases: 0 residuals, 1 factor (W, Phi_u, S_ii), 2 factor chain, 3 solve
right-hand side and Phi^-1, 4 forward chain, 5 backward chain, 6 dx / dz / ds finish, 7 refinement
residuals, 8 step lengths / sigma / update. Cycles of one QP (lane 0 of its wave), per iteration.
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "ab", os.environ.get("GPROF_LIB", "libsrbd_mpc_gprof.so"))
NAMES = ["residuals", "factor: W, Phi_u, S_ii", "factor: chain", "solve: rhs, Phi^-1", "solve: fwd chain",
         "solve: bwd chain", "solve: finish", "refine residuals", "steps / update"]


def build():
    from biped_pympc_amd.build import HIPCC, LIB_DIR, unit_compile_cmd
    obj = "/tmp/srbd_mpc_gprof.o"
    subprocess.run(unit_compile_cmd("srbd_mpc.hip", ["-include", os.path.join(ROOT, "scripts", "phase_prof.hpp"),
                                                      "-fPIC", "-c", "-o", obj]), check=True)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", LIB, obj,
                    os.path.join(LIB_DIR, "srbd_reg20.o"), os.path.join(LIB_DIR, "srbd_regN.o")], check=True)
    print(LIB)


def run(N=10, B=96, K=5):
    os.environ["SRBD_LIB"] = LIB
    import torch
    from biped_pympc_amd import _native, solver
    from biped_pympc_amd.utils.synthetic import make_workload, solver_init
    L = _native.lib()
    L.srbd_debug_phase_cycles.argtypes = [ctypes.c_void_p]
    wl = make_workload(B, N, seed=77)
    ins = [torch.from_numpy(a).cuda() for a in wl.inputs]
    H, f, A, b, G, d = solver.qp_former(ins, N)
    it = [torch.from_numpy(a).cuda() for a in solver_init(d.cpu().numpy(), N)]
    qp = [H, G, A, f, d, b]
    acc = (ctypes.c_ulonglong * 16)()
    with _native.solver_path("general"):
        solver.pdipm(qp, it, N, K)
        torch.cuda.synchronize()
        L.srbd_debug_phase_cycles(acc)  # reset
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        solver.pdipm(qp, it, N, K)
        e1.record()
        e1.synchronize()
    L.srbd_debug_phase_cycles(acc)
    tot = sum(acc[k] for k in range(len(NAMES)))
    print(f"general path N={N} B={B} K={K}: {e0.elapsed_time(e1):.3f} ms; cycles per QP per iteration:")
    for k, n in enumerate(NAMES):
        c = acc[k] / B / K
        print(f"  {n:28s} {c:12.0f}  ({100.0 * acc[k] / max(tot, 1):5.1f} %)")
    print(f"  {'total':28s} {tot / B / K:12.0f}")


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        run(*[int(v) for v in sys.argv[2:5]])
