"""Fused-step A/B of compile-time variants on one GPU box (the bench's own kernel and timing).

python scripts/variant_bench.py [--horizon N] [--rounds R] [--batch B] NAME=FLAGS [NAME=FLAGS ...]
Each variant is built from the working tree's csrc with its -D flags into /tmp/libsrbd_mpc_<NAME>.so;
the variants then run bench.py (--steps 50, SRBD_LIB) in turn, R rounds, and the fused kernel's
HIP-event time per launch is printed per run and as the per-variant median.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--horizon", type=int, default=10)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("variants", nargs="+")
    a = p.parse_args()
    libs = {}
    for spec in a.variants:
        name, _, flags = spec.partition("=")
        lib = f"/tmp/libsrbd_mpc_{name}.so"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        *flags.split(), "-I", os.path.join(ROOT, "include"), "-o", lib,
                        os.path.join(ROOT, "biped_pympc_amd/csrc/srbd_mpc.hip")], check=True)
        libs[name] = lib
    res = {n: [] for n in libs}
    for _ in range(a.rounds):
        for name, lib in libs.items():
            r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "50", "--warmup", "10",
                                "--no-cpu-baseline", "--horizon", str(a.horizon),
                                "--batch-per-gpu", str(a.batch)],
                               env={**os.environ, "SRBD_LIB": lib}, capture_output=True, text=True, timeout=300)
            if r.returncode:
                raise SystemExit(f"{name}: bench failed\n{r.stderr[-2000:]}")
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res[name].append(d["kernels_ms"]["mpc_step_fused"])
            print(f"{name:12s} {res[name][-1]:.4f} ms", flush=True)
    for name, v in res.items():
        print(f"median {name:12s} {statistics.median(v):.4f} ms")


if __name__ == "__main__":
    main()
