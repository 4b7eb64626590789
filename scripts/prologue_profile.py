"""Diagnostic: shader-clock cycles of the fused kernel's prologue and epilogue per QP (GPU box).

Builds a PATCHED COPY of csrc with scripts/phase_prof.hpp force-included (the product sources are not touched) whose
extra stamps split the work before the Newton loop into: input read + former model, stage-block
and f/b/d set-up, per-QP constants (C, K0, K1, slot tables), iterate init; and the work after it
(outputs). The Newton iterations themselves are stamped as in scripts/phase_profile.py.
    python scripts/prologue_profile.py [N] [B] [K]
"""
import ctypes
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "ab", "libsrbd_mpc_prologue.so")  # built on the CPU host (ab/ is not in git)


def patch(src: str) -> str:
    def rep(old, new):
        nonlocal src
        assert src.count(old) == 1, old
        src = src.replace(old, new)
    rep("  C.lane = lane;\n", "  C.lane = lane;\n  PROF_MARK_CTX(C);\n")
    rep("    former_model(F, P, lane);\n", "    former_model(F, P, lane);\n    PROF_ADD_CTX(C, 8);\n")
    rep("  // ---- per-QP constants ----\n", "  PROF_ADD_CTX(C, 9);\n  // ---- per-QP constants ----\n")
    rep("  // ---- iterate ----\n", "  PROF_ADD_CTX(C, 10);\n  // ---- iterate ----\n")
    rep("  PROF_MARK_CTX(C);\n  const int n_iter", "  PROF_ADD_CTX(C, 11);\n  const int n_iter")
    rep("  PROF_FLUSH(C);\n  auto outp", "  PROF_ADD_CTX(C, 7);\n  auto outp")
    # epilogue stamp + the single flush at the very end of the body
    i = src.index("// 2 waves per SIMD: 2 one-wave QPs")
    j = src.rindex("}\n", 0, i)
    src = src[:j] + "  PROF_ADD_CTX(C, 12);\n  PROF_FLUSH(C);\n" + src[j:]
    return src


def build():
    with tempfile.TemporaryDirectory() as td:
        d = os.path.join(td, "biped_pympc_amd", "csrc")  # srbd_mpc.hip includes ../../include/srbd_mpc.h
        shutil.copytree(os.path.join(ROOT, "biped_pympc_amd", "csrc"), d)
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(td, "include"))
        p = os.path.join(d, "pdipm_srbd_reg.hpp")
        src = patch(open(p).read())
        open(p, "w").write(src)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-include", os.path.join(ROOT, "scripts", "phase_prof.hpp"), "-I", os.path.join(ROOT, "include"), "-o", LIB,
                        os.path.join(d, "srbd_mpc.hip")], check=True)


def main():
    if not os.path.exists(LIB) or "--rebuild" in sys.argv:
        build()
    os.environ["SRBD_LIB"] = LIB
    import torch
    from biped_pympc_amd import _native, solver
    from biped_pympc_amd.utils.synthetic import make_workload
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    N = int(args[0]) if args else 10
    B = int(args[1]) if len(args) > 1 else 4096
    K = int(args[2]) if len(args) > 2 else 10
    L = _native.lib()
    L.srbd_debug_phase_cycles.argtypes = [ctypes.c_void_p]
    wl = make_workload(B, N, seed=1)
    ins = [torch.from_numpy(a).cuda() for a in wl.inputs]
    bufs = solver.MPCSolveBuffers.allocate(N, B)
    solver.mpc_solve(ins, N, K, buffers=bufs)
    torch.cuda.synchronize()
    acc = (ctypes.c_ulonglong * 16)()
    L.srbd_debug_phase_cycles(acc)  # reset
    solver.mpc_solve(ins, N, K, buffers=bufs)
    torch.cuda.synchronize()
    L.srbd_debug_phase_cycles(acc)
    names = {8: "input read + former model", 9: "stage blocks, G, f/b/d set-up", 10: "per-QP constants",
             11: "iterate init", 0: "iterations: residuals", 1: "iterations: factor build",
             2: "iterations: factor chain", 3: "iterations: solve parallel parts", 4: "iterations: chains",
             5: "iterations: steps / update", 6: "iterations: refinement residual", 7: "last-iteration tail",
             12: "outputs (epilogue)"}
    tot = sum(acc[k] for k in names)
    print(f"N={N} B={B} K={K}: cycles per QP (one wave's wall clock, s_memtime)")
    for k in (8, 9, 10, 11, 0, 1, 2, 3, 4, 5, 6, 7, 12):
        print(f"  {names[k]:34s} {acc[k] / B:10.0f}  ({100 * acc[k] / tot:5.1f} %)")
    print(f"  {'total':34s} {tot / B:10.0f}")


if __name__ == "__main__":
    main()
