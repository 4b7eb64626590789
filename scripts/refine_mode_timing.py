"""Fused-step kernel time (HIP events) in both affine-refinement modes, alternating, B = 4096, K = 10,
at N = 10 and N = 20 (srbd_set_refinement: 0 adaptive, 1 every iteration).

    python scripts/refine_mode_timing.py   -> one JSON line per (N, mode, round)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biped_pympc_amd import _native, solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload  # noqa: E402


def ms(fn, reps=50, warm=10):
    for _ in range(warm):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


for N in (10, 20):
    B, K = 4096, 10
    ins = [torch.from_numpy(a).cuda() for a in make_workload(B, N, seed=1000).inputs]
    bufs = solver.MPCSolveBuffers.allocate(N, B, "cuda")
    for r in range(3):
        for mode in ("adaptive", "every_iteration"):
            with _native.refinement(mode):
                t = ms(lambda: solver.mpc_solve(ins, N, K, 1.0, buffers=bufs))
            print(json.dumps({"N": N, "mode": mode, "round": r, "ms": round(t, 4), "solves_per_s": round(B / t * 1e3, 1)}), flush=True)
