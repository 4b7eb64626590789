"""A/B of the solver kernels on one workload: time per launch (HIP events on the launch stream)
and agreement of the results. Run on the GPU box: python scripts/kernel_ab.py [N] [B] [K]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from biped_pympc_amd import _native, solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
paths = sys.argv[4].split(",") if len(sys.argv) > 4 else ["auto", "lds", "general"]

wl = make_workload(B, N, seed=1)
inputs = [torch.from_numpy(a).cuda() for a in wl.inputs]
qp = solver.qp_former(inputs, N)
sol_qp = [qp[0], qp[4], qp[2], qp[1], qp[5], qp[3]]
res = {}
for path in paths:
    with _native.solver_path(path):
        out = solver.pdipm(sol_qp, None, N, K, 1.0)
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record(s)
        for _ in range(reps):
            solver.pdipm(sol_qp, None, N, K, 1.0, outputs=out)
        e1.record(s)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
    res[path] = [o.cpu().numpy() for o in out]
    print(f"{path:8s} N={N} B={B} K={K}: {ms:.4f} ms/launch  {B / ms * 1e3:,.0f} solves/s")
base = paths[0]
for path in paths[1:]:
    errs = []
    for k in range(4):
        a, b = res[base][k], res[path][k]
        errs.append(float((np.abs(a - b).max(axis=1) / np.maximum(np.abs(b).max(axis=1), 1e-300)).max()))
    print(f"{base} vs {path}: worst-env rel diff x,s,z,y = " + ", ".join(f"{e:.2e}" for e in errs))
