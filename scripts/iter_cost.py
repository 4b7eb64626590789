"""Diagnostic: fused-step time vs Newton iteration count (the intercept of the line is prologue + epilogue) at
B = 4096, N = 10 and 20: the per-iteration slope and the fixed cost. Run on the GPU box."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from biped_pympc_amd import solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload  # noqa: E402

for N in (10, 20):
    B = 4096
    wl = make_workload(B, N, seed=1)
    ins = [torch.from_numpy(a).cuda() for a in wl.inputs]
    bufs = solver.MPCSolveBuffers.allocate(N, B)
    for K in (1, 2, 3, 5, 10):
        for _ in range(3):
            solver.mpc_solve(ins, N, K, buffers=bufs)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            solver.mpc_solve(ins, N, K, buffers=bufs)
        e1.record()
        torch.cuda.synchronize()
        print(f"N={N} K={K:2d}: {e0.elapsed_time(e1) / 20:.4f} ms", flush=True)
