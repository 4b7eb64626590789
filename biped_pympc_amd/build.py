"""Build the native libraries in-tree (hipcc for gfx950 + gcc for the thin CusADi-ABI shims).

Outputs (biped_pympc_amd/lib/):
  libsrbd_mpc.so                                  HIP kernels + extended C-ABI (include/srbd_mpc.h)
  libqp_former.so                                 CusADi `evaluate` for 'qp_former' (N = 10)
  libsparse_pdipm_multiple_iterations.so          CusADi `evaluate` for the deployed solver (N=10, 5 it)
  libqp_former_N<N>.so, libsparse_pdipm_multiple_iterations_N<N>_K<K>.so   other configurations
Replaces the reference's CasADi -> CUDA codegen + CMake pipeline (run_codegen.py:9-44), which
takes ~3 h for 5 unrolled Newton iterations (README.md:80-84); this builds in seconds.
"""
from __future__ import annotations

import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB_DIR = os.path.join(PKG, "lib")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SRBD_OFFLOAD_ARCH", "gfx950")

# (function name, N, K) of the thin CusADi-ABI libraries to build
DROPIN_CONFIGS = [
    ("qp_former", 10, None),
    ("sparse_pdipm_multiple_iterations", 10, 5),
    ("qp_former", 20, None),
    ("sparse_pdipm_multiple_iterations", 10, 10),
    ("sparse_pdipm_multiple_iterations", 20, 10),
]


def dropin_lib_name(fn: str, N: int, K: int | None) -> str:
    if fn == "qp_former":
        return "libqp_former.so" if N == 10 else f"libqp_former_N{N}.so"
    if N == 10 and K == 5:
        return "libsparse_pdipm_multiple_iterations.so"
    return f"libsparse_pdipm_multiple_iterations_N{N}_K{K}.so"


def _newer(target: str, sources: list[str]) -> bool:
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(s) <= t for s in sources)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _build_dropin_lib(fn: str, N: int, K: int | None, core: str, force: bool, verbose: bool) -> str:
    shim = os.path.join(CSRC, "dropin_evaluate.c")
    out = os.path.join(LIB_DIR, dropin_lib_name(fn, N, K))
    if not force and _newer(out, [shim, core, os.path.join(INCLUDE, "srbd_mpc.h")]):
        return out
    defs = ["-DSRBD_FN_FORMER"] if fn == "qp_former" else ["-DSRBD_FN_PDIPM", f"-DSRBD_ITERS={K}"]
    cmd = ["gcc", "-O2", "-fPIC", "-shared", f"-DSRBD_N={N}", *defs, "-o", out, shim,
           f"-L{LIB_DIR}", "-lsrbd_mpc", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd))
    _run(cmd)
    return out


def build_dropin(kind: str, N: int, K: int | None) -> str:
    """Thin CusADi-ABI library for one (function, horizon, iterations) configuration."""
    fn = "qp_former" if kind == "qp_former" else "sparse_pdipm_multiple_iterations"
    core = build()
    return _build_dropin_lib(fn, N, K, core, False, False)


# the two HIP translation units of libsrbd_mpc.so and their unit-specific flags: the N = 20 register
# kernels in their own unit, scheduled with the register-pressure trackers (csrc/reg20.hpp)
HIP_UNITS = {
    "srbd_mpc.hip": ["-DSRBD_SPLIT_REG20"],
    "srbd_reg20.hip": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
    "srbd_regN.hip": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],  # the other register horizons
}


def unit_compile_cmd(unit: str, extra: list[str]) -> list[str]:
    """hipcc command line of one translation unit exactly as the product build compiles it (the
    ISA audit, tests/test_isa_hazards.py, appends --cuda-device-only -S to the same flags)."""
    return [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", *HIP_UNITS[unit], *extra,
            os.path.join(CSRC, unit)]


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    core = os.path.join(LIB_DIR, "libsrbd_mpc.so")
    # the translation unit and every header it includes (csrc/*.hpp)
    srcs = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith((".hip", ".hpp"))]
    srcs.append(os.path.join(INCLUDE, "srbd_mpc.h"))
    if force or not _newer(core, srcs):
        # the N = 20 register kernels in their own unit, scheduled with the register-pressure
        # trackers (csrc/reg20.hpp), linked into the same library
        objs = [os.path.join(LIB_DIR, u.replace(".hip", ".o")) for u in HIP_UNITS]
        units = [unit_compile_cmd(u, ["-fPIC", "-c", "-o", o]) for u, o in zip(HIP_UNITS, objs)]
        for cmd in units:
            if verbose:
                print(" ".join(cmd))
        # the units compile in parallel (independent translation units)
        procs = [subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for cmd in units]
        for cmd, pr in zip(units, procs):
            out, err = pr.communicate()
            if pr.returncode != 0:
                raise RuntimeError(f"build failed: {' '.join(cmd)}\n{out}\n{err}")
        link = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", core, *objs]
        if verbose:
            print(" ".join(link))
        _run(link)
    for fn, N, K in DROPIN_CONFIGS:
        _build_dropin_lib(fn, N, K, core, force, verbose)
    return core


if __name__ == "__main__":
    print(build(force=True, verbose=True))
