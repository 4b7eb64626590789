"""Diagnostic (GPU box): per-iteration error of one env of a stress workload (tests/_stress.py)
for each solver path vs the oracle, and the dense-LU restatement vs the oracle.
    python scripts/diag_stress_env.py tilt_N10 11 [KMAX]"""
import sys

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from biped_pympc_amd import _native, solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import solver_init  # noqa: E402
from oracle import oracle  # noqa: E402
from oracle.pdipm_dense import pdipm_dense  # noqa: E402
from tests._stress import stress_workload  # noqa: E402

name, e = sys.argv[1], int(sys.argv[2])
KMAX = int(sys.argv[3]) if len(sys.argv) > 3 else 20
N, wl = stress_workload(name)
H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
it = solver_init(d, N, y0=1.0)
cu = lambda a: [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in a]  # noqa: E731
qp = cu([H, G, A, f, d, b])
dn = [t[e] for t in it]
rel = lambda o, r: float(np.abs(o - r).max() / max(np.abs(r).max(), 1e-300))  # noqa: E731
for K in range(1, KMAX + 1):
    ref = oracle.pdipm(N, K, [H, G, A, f, d, b, *it])
    dn = pdipm_dense(N, 1, H[e], G[e], A[e], f[e], d[e], b[e], *dn[:4])
    line = [f"K={K:2d}", "dense " + " ".join(f"{v}{rel(dn[k], ref[k][e]):.0e}" for k, v in enumerate("xszy"))]
    for path in ("auto", "general", "lds"):
        with _native.solver_path(path):
            o = solver.pdipm(qp, cu(list(it)), N, K)
            torch.cuda.synchronize()
        o = [t.cpu().numpy()[e] for t in o]
        line.append(f"{path} " + " ".join(f"{v}{rel(o[k], ref[k][e]):.0e}" for k, v in enumerate("xszy")))
    mu = ref[5][e, 0] if ref[5].ndim > 1 else ref[5][e]
    line.append(f"mu {float(mu):.1e} zmin {ref[2][e].min():.1e} smin {ref[1][e].min():.1e}")
    print(" | ".join(line), flush=True)
