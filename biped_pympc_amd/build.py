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

import hashlib
import os
import re
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


_ID_RE = re.compile(rb"srbd-(build|shim)-id:([0-9a-f]{16})")


def embedded_id(path: str) -> str | None:
    """The build id a library carries ("srbd-build-id:<16 hex>" in libsrbd_mpc.so's read-only data,
    "srbd-shim-id:<16 hex>" in a drop-in), read from the file without loading it; None if absent."""
    try:
        with open(path, "rb") as fh:
            m = _ID_RE.search(fh.read())
    except OSError:
        return None
    return m.group(2).decode() if m else None


def _digest(parts) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(p if isinstance(p, bytes) else str(p).encode())
        h.update(b"\0")
    return h.hexdigest()[:16]


def core_sources() -> list[str]:
    """Every file libsrbd_mpc.so is compiled from: the HIP units, their headers, the C-ABI header."""
    srcs = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith((".hip", ".hpp"))]
    return srcs + [os.path.join(INCLUDE, "srbd_mpc.h")]


def source_hash(sources: list[str] | None = None) -> str:
    """Build id of libsrbd_mpc.so: sha256 over the sources' names and bytes and the compile flags,
    truncated to 16 hex digits. Embedded in the library (srbd_build_id()); build() rebuilds when the
    library's id differs from this, whatever the files' mtimes say."""
    parts = [ARCH, repr(sorted(HIP_UNITS.items())), repr(_COMMON_FLAGS)]
    for s in core_sources() if sources is None else sources:
        parts += [os.path.basename(s), open(s, "rb").read()]
    return _digest(parts)


def _unit_hash(unit: str, bid: str) -> str:
    """What one object file depends on: its unit, every header (csrc/*.hpp, include/srbd_mpc.h), the
    flags, and -- for the main unit, which embeds it -- the library's build id."""
    parts = [ARCH, unit, repr(HIP_UNITS[unit]), repr(_COMMON_FLAGS), bid if unit == "srbd_mpc.hip" else ""]
    for s in core_sources():
        if s.endswith(".hip") and os.path.basename(s) != unit:
            continue
        if s.endswith(".h") and unit != "srbd_mpc.hip":  # only the main unit includes the C-ABI header
            continue
        parts += [os.path.basename(s), open(s, "rb").read()]
    return _digest(parts)


def _shim_hash(fn: str, N: int, K: int | None, core_id: str) -> str:
    shim = os.path.join(CSRC, "dropin_evaluate.c")
    return _digest([fn, N, K, core_id, open(shim, "rb").read(), open(os.path.join(INCLUDE, "srbd_mpc.h"), "rb").read()])


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _build_dropin_lib(fn: str, N: int, K: int | None, core: str, force: bool, verbose: bool) -> str:
    shim = os.path.join(CSRC, "dropin_evaluate.c")
    out = os.path.join(LIB_DIR, dropin_lib_name(fn, N, K))
    sid = _shim_hash(fn, N, K, embedded_id(core) or "")
    if not force and embedded_id(out) == sid:
        return out
    defs = ["-DSRBD_FN_FORMER"] if fn == "qp_former" else ["-DSRBD_FN_PDIPM", f"-DSRBD_ITERS={K}"]
    cmd = ["gcc", "-O2", "-fPIC", "-shared", f"-DSRBD_N={N}", *defs, f'-DSRBD_SHIM_ID="{sid}"', "-o", out, shim,
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


_COMMON_FLAGS = ["-O3", "-std=c++17"]


def unit_compile_cmd(unit: str, extra: list[str]) -> list[str]:
    """hipcc command line of one translation unit exactly as the product build compiles it (the
    ISA audit, tests/test_isa_hazards.py, appends --cuda-device-only -S to the same flags)."""
    return [HIPCC, f"--offload-arch={ARCH}", *_COMMON_FLAGS, *HIP_UNITS[unit], *extra,
            os.path.join(CSRC, unit)]


def _compile_parallel(cmds: list[list[str]]) -> None:
    """Run independent compiles at once; on any failure the others are killed and reaped before
    raising, so no orphan keeps writing objects into lib/."""
    procs = [subprocess.Popen(c, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for c in cmds]
    failed = None
    try:
        for c, pr in zip(cmds, procs):
            out, err = pr.communicate()
            if pr.returncode != 0:
                failed = f"build failed: {' '.join(c)}\n{out}\n{err}"
                break
    finally:
        for pr in procs:
            if pr.poll() is None:
                pr.kill()
            pr.wait()
    if failed:
        raise RuntimeError(failed)


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    core = os.path.join(LIB_DIR, "libsrbd_mpc.so")
    bid = source_hash()
    if force or embedded_id(core) != bid:
        objs = [os.path.join(LIB_DIR, u.replace(".hip", ".o")) for u in HIP_UNITS]
        # srbd_build_id() is defined in the main unit; the id names the sources and flags of all units.
        # An object is reused when its sidecar records the hash of exactly what it was compiled from.
        stale = []
        for u, o in zip(HIP_UNITS, objs):
            uh = _unit_hash(u, bid)
            try:
                same = not force and open(o + ".id").read().strip() == uh and os.path.exists(o)
            except OSError:
                same = False
            if not same:
                stale.append((u, o, uh))
        units = [unit_compile_cmd(u, ["-fPIC", "-c", *([f'-DSRBD_BUILD_ID="{bid}"'] if u == "srbd_mpc.hip" else []),
                                      "-o", o]) for u, o, _ in stale]
        for cmd in units:
            if verbose:
                print(" ".join(cmd))
        for _, o, _ in stale:
            if os.path.exists(o + ".id"):
                os.remove(o + ".id")
        _compile_parallel(units)  # independent translation units
        for _, o, uh in stale:
            with open(o + ".id", "w") as fh:
                fh.write(uh + "\n")
        tmp = core + ".tmp"
        link = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", tmp, *objs]
        if verbose:
            print(" ".join(link))
        _run(link)
        os.replace(tmp, core)  # a process that has the old library mapped keeps its copy
        if embedded_id(core) != bid:
            raise RuntimeError(f"{core}: build id {embedded_id(core)} != source hash {bid}")
    for fn, N, K in DROPIN_CONFIGS:
        _build_dropin_lib(fn, N, K, core, force, verbose)
    return core


if __name__ == "__main__":
    print(build(force=True, verbose=True))
