"""GPU: worst-env parity of the HIP solver vs the oracle (and dense LU vs oracle) per K."""
import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from biped_pympc_amd import solver
from biped_pympc_amd.utils.synthetic import make_workload, solver_init
from oracle import oracle
from oracle.pdipm_dense import pdipm_dense
from tests._util import rel_err_rows
def cuda(a): return [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in a]
names = ["x", "s", "z", "y"]
for N, gait in ((10, False), (10, True), (20, False), (20, True)):
    wl = make_workload(64, N, seed=101, random_gait=gait)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    it = solver_init(d, N)
    for K in (1, 5, 10, 20):
        ref = oracle.pdipm(N, K, [H, G, A, f, d, b, *it])
        o = solver.pdipm(cuda([H, G, A, f, d, b]), cuda(list(it)), N, K)
        torch.cuda.synchronize()
        o = [t.cpu().numpy() for t in o]
        e = [rel_err_rows(o[k], ref[k]) for k in range(4)]
        ne = 8 if N == 10 else 4
        den = [np.stack(v) for v in zip(*[pdipm_dense(N, K, H[i], G[i], A[i], f[i], d[i], b[i], *(t[i] for t in it)) for i in range(ne)])]
        dd = [rel_err_rows(den[k], ref[k][:ne]).max() for k in range(4)]
        print(f"N={N} gait={gait} K={K:2d} gpu " + " ".join(f"{names[k]} {e[k].max():.1e}/{np.median(e[k]):.0e}" for k in range(4))
              + " | dense(8) " + " ".join(f"{names[k]} {dd[k]:.1e}" for k in range(4)), flush=True)
