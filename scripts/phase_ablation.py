"""Diagnostic: marginal cost of each solver phase in the real (2 waves/SIMD) context.

Builds variants of libsrbd_mpc.so with -DSRBD_REPEAT_PHASE=k (k = 1 residuals, 2 factorisation, 4 its S_ii build,
3 affine solve: each idempotent, run twice per Newton iteration) into /tmp and times the N=10
solver launch with each; the difference to the base build is that phase's cost per launch.
Run on the GPU box: python scripts/phase_ablation.py [N] [B] [K]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
names = {0: "base", 1: "residuals", 2: "factorisation (parallel + chain)", 4: "factorisation: S_ii build only",
         3: "one solve (parallel + chains)"}
res = {}
for k in names:
    lib = f"/tmp/libsrbd_mpc_rep{k}.so"
    flags = [] if k == 0 else [f"-DSRBD_REPEAT_PHASE={k}"]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", *flags,
                    "-o", lib, os.path.join(ROOT, "biped_pympc_amd/csrc/srbd_mpc.hip")], check=True)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts/kernel_ab.py"), str(N), str(B), str(K), "auto"],
                         env={**os.environ, "SRBD_LIB": lib}, capture_output=True, text=True, check=True).stdout
    ms = float([l for l in out.splitlines() if "ms/launch" in l][0].split(":")[1].split("ms")[0])
    res[k] = ms
    print(f"{names[k]:36s} {ms:8.4f} ms/launch" + ("" if k == 0 else f"   marginal {ms - res[0]:7.4f} ms"
                                                       f" ({100 * (ms - res[0]) / res[0]:5.1f} %)"), flush=True)
