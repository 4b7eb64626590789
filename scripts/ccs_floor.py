"""CPU: dense-LU restatement vs the C oracle after K iterations from the _ccs init (x_init random, y = 0):
the FP64 floor under tests/test_gpu_parity.py::test_ccs_entry_from_arbitrary_x_init."""
import sys, numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biped_pympc_amd import layout
from biped_pympc_amd.utils.synthetic import make_workload
from oracle import oracle
from oracle.pdipm_dense import pdipm_dense
from tests._util import rel_err_rows
for N in (10, 20, 5):
    for K in (1, 10):
        B = 48
        wl = make_workload(B, N, seed=700 + N + K, random_gait=True)
        H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
        dims = layout.Dims(N)
        x0 = np.random.default_rng(N + K).normal(0, 5.0, (B, dims.nz))
        Gd = layout.to_dense(G, *layout.ccs_G(N), (dims.n_ineq, dims.nz))
        s0 = np.maximum(d - np.einsum("bij,bj->bi", Gd, x0), 1.0)
        it = [x0, s0, np.ones((B, dims.n_ineq)), np.zeros((B, dims.n_eq))]
        ref = oracle.pdipm(N, K, [H, G, A, f, d, b, *it])
        ne = 12 if N <= 10 else 6
        den = [np.stack(v) for v in zip(*[pdipm_dense(N, K, H[e], G[e], A[e], f[e], d[e], b[e], *(t[e] for t in it)) for e in range(ne)])]
        print(N, K, " ".join(f"{rel_err_rows(den[k], ref[k][:ne]).max():.1e}" for k in range(4)), flush=True)
