"""Build a compile-time variant of libsrbd_mpc.so (all three translation units, same flags as
biped_pympc_amd/build.py plus the given flags) into OUT, on the CPU host.

    python scripts/build_variant.py OUT [--no-regn] [-DFLAG | compiler flag ...]

--reg20=FLAG adds FLAG to the N = 20 unit only (e.g. --reg20=-include --reg20=scripts/phase_prof.hpp:
the phase stamps of the N = 20 kernels, whose accumulators then live in that unit alone).
--no-regn links scripts/regn_stub.hip instead of the srbd_regN.hip unit (1 min instead of 7): the
horizons other than 10 and 20 then run the LDS-resident kernels (N = 10 / 20 experiments only).

Diagnostic tool: the product library is only ever built by biped_pympc_amd/build.py.
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "biped_pympc_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def build_variant(out: str, flags: list[str], regn: bool = True, reg20_flags: list[str] = ()) -> str:
    with tempfile.TemporaryDirectory() as td:
        o20, on, om = (os.path.join(td, n) for n in ("reg20.o", "regN.o", "main.o"))
        base = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "-I", os.path.join(ROOT, "include"),
                *flags]
        trk = ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"]
        procs = [subprocess.Popen(base + trk + list(reg20_flags) + ["-o", o20, os.path.join(CSRC, "srbd_reg20.hip")]),
                 subprocess.Popen(base + (trk + ["-o", on, os.path.join(CSRC, "srbd_regN.hip")] if regn else
                                          ["-o", on, os.path.join(ROOT, "scripts", "regn_stub.hip")])),
                 subprocess.Popen(base + ["-DSRBD_SPLIT_REG20", "-o", om, os.path.join(CSRC, "srbd_mpc.hip")])]
        if any(p.wait() for p in procs):
            raise SystemExit("variant compile failed")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out, om, o20, on], check=True)
    return out


if __name__ == "__main__":
    args = sys.argv[2:]
    r20 = [a[len("--reg20="):] for a in args if a.startswith("--reg20=")]
    rest = [a for a in args if a != "--no-regn" and not a.startswith("--reg20=")]
    print(build_variant(sys.argv[1], rest, regn="--no-regn" not in args, reg20_flags=r20))
