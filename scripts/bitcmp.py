"""Diagnostic: dump the fused step's solution (N = 10, 20; standing and randomized gait; K = 1, 10, 20)
with the library SRBD_LIB points at, or compare two such dumps bit for bit.

    SRBD_LIB=ab/libsrbd_mpc_old.so python scripts/bitcmp.py dump gpurun_out/old.npz
    python scripts/bitcmp.py dump gpurun_out/new.npz
    python scripts/bitcmp.py cmp gpurun_out/old.npz gpurun_out/new.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(path):
    import torch
    from biped_pympc_amd import solver
    from biped_pympc_amd.utils.synthetic import make_workload
    out = {}
    for N in (10, 20):
        for gait in (False, True):
            wl = make_workload(512, N, seed=900 + N + gait, random_gait=gait)
            ins = [torch.from_numpy(a).cuda() for a in wl.inputs]
            for K in (1, 10, 20):
                res = solver.mpc_solve(ins, N, K, 1.0)
                torch.cuda.synchronize()
                for k, name in enumerate(("x", "s", "z", "y", "res", "mu")):
                    out[f"N{N}_g{int(gait)}_K{K}_{name}"] = res[k].cpu().numpy()
    np.savez(path, **out)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    worst = 0.0
    for k in A.files:
        x, y = A[k], B[k]
        same = np.array_equal(x.view(np.uint64), y.view(np.uint64))
        d = float(np.max(np.abs(x - y)) / max(np.max(np.abs(x)), 1e-300))
        worst = max(worst, d)
        if not same:
            print(f"{k}: differs, max rel {d:.3e}")
    print(f"{len(A.files)} arrays, worst rel diff {worst:.3e}" + (" (bit-identical)" if worst == 0 else ""))


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        cmp(sys.argv[2], sys.argv[3])
