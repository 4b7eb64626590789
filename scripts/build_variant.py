"""Build a compile-time variant of libsrbd_mpc.so (both translation units, same flags as
biped_pympc_amd/build.py plus the given -D flags) into OUT, on the CPU host.

    python scripts/build_variant.py OUT [-DFLAG ...]

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
        o20, om = os.path.join(td, "reg20.o"), os.path.join(td, "main.o")
        base = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", *flags]
        subprocess.run(base + ["-mllvm", "-amdgpu-use-amdgpu-trackers=1", "-o", o20,
                               os.path.join(CSRC, "srbd_reg20.hip")], check=True)
        subprocess.run(base + ["-DSRBD_SPLIT_REG20", "-o", om, os.path.join(CSRC, "srbd_mpc.hip")], check=True)
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out, om, o20], check=True)
    return out


if __name__ == "__main__":
    print(build_variant(sys.argv[1], sys.argv[2:]))
