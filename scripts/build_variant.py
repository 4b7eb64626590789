"""Build a compile-time variant of libsrbd_mpc.so (all three translation units, same flags as
biped_pympc_amd/build.py plus the given flags) into OUT, on the CPU host.

    python scripts/build_variant.py OUT [-DFLAG | compiler flag ...]

Diagnostic tool: the product library is only ever built by biped_pympc_amd/build.py.
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "biped_pympc_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def build_variant(out: str, flags: list[str]) -> str:
    with tempfile.TemporaryDirectory() as td:
        o20, on, om = (os.path.join(td, n) for n in ("reg20.o", "regN.o", "main.o"))
        base = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "-I", os.path.join(ROOT, "include"),
                *flags]
        trk = ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"]
        procs = [subprocess.Popen(base + trk + ["-o", o20, os.path.join(CSRC, "srbd_reg20.hip")]),
                 subprocess.Popen(base + trk + ["-o", on, os.path.join(CSRC, "srbd_regN.hip")]),
                 subprocess.Popen(base + ["-DSRBD_SPLIT_REG20", "-o", om, os.path.join(CSRC, "srbd_mpc.hip")])]
        if any(p.wait() for p in procs):
            raise SystemExit("variant compile failed")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out, om, o20, on], check=True)
    return out


if __name__ == "__main__":
    print(build_variant(sys.argv[1], sys.argv[2:]))
