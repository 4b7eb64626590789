import sys, numpy as np
from biped_pympc_amd.utils.synthetic import make_workload, solver_init
from oracle import oracle
from oracle.pdipm_dense import pdipm_dense
from tests._util import rel_err_rows
N, seed, gait = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3] == "1"
wl = make_workload(64, N, seed=seed, random_gait=gait)
H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
it = solver_init(d, N)
for K in (10, 20):
    ref = oracle.pdipm(N, K, [H, G, A, f, d, b, *it])
    den = [np.stack(v) for v in zip(*[pdipm_dense(N, K, H[i], G[i], A[i], f[i], d[i], b[i], *(t[i] for t in it)) for i in range(64)])]
    e = np.max([rel_err_rows(den[k], ref[k]) for k in range(4)], axis=0)
    print(f"N={N} seed={seed} gait={gait} K={K}: dense-vs-oracle worst {e.max():.1e} (env {e.argmax()}), median {np.median(e):.1e}", flush=True)
