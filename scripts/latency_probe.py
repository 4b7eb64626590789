"""Small-batch latency of the fused step across horizons (one-wave QPs at N <= 10, two-wave from N = 11):
whether more waves per QP shorten one QP's solve when the chip is mostly idle (B << 2048 resident slots).

    python scripts/latency_probe.py  -> one JSON object per line: N, B, K, ms per launch (HIP events)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biped_pympc_amd import solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload  # noqa: E402


def ms(fn, reps=200, warm=20):
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


for N in (8, 9, 10, 11, 12):
    for B in (1, 64, 256, 1024, 4096):
        wl = make_workload(B, N, seed=5)
        ins = [torch.from_numpy(a).cuda() for a in wl.inputs]
        bufs = solver.MPCSolveBuffers.allocate(N, B, "cuda")
        for K in (5, 10):
            t = ms(lambda: solver.mpc_solve(ins, N, K, 1.0, buffers=bufs), reps=50 if B >= 1024 else 200)
            print(json.dumps({"N": N, "B": B, "K": K, "ms": round(t, 4)}), flush=True)
