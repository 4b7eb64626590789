"""Generate tests/golden/dense_floor_ragged.npz (committed fixture; CPU, ~2 min on 8 cores).

For each ragged-batch workload of tests/test_gpu_parity.py::test_ragged_batches (N in {10, 20},
B in {1, 3, 13, 509}, randomized gait, K = 10 iterations from the GPU caller's init), the per-env
relative x error between the two independent CPU restatements of the solver -- the C oracle
(sparse LDL^T) and oracle/pdipm_dense.py (dense LU of the full KKT). That spread is the FP64
floor of the comparison: an env whose two exact eliminations already disagree by 1e-7 cannot be
asked to match either one closer than that. The GPU test allows max(tol, 4 x floor) per env.
"""
import os
import sys
from multiprocessing import Pool

os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import numpy as np  # noqa: E402

from biped_pympc_amd.utils.synthetic import make_workload, solver_init  # noqa: E402
from oracle import oracle  # noqa: E402
from oracle.pdipm_dense import pdipm_dense  # noqa: E402
from tests._util import rel_err_rows  # noqa: E402

K = 10
CASES = [(N, B) for N in (10, 20) for B in (1, 3, 13, 509)]


def workload(N, B):
    wl = make_workload(B, N, seed=4000 + B, random_gait=True, residuals=True)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    return wl, (H, f, A, b, G, d), solver_init(d, N, y0=1.0)


def one(args):
    N, B, e = args
    _, (H, f, A, b, G, d), it = workload(N, B)
    return pdipm_dense(N, K, H[e], G[e], A[e], f[e], d[e], b[e], *(t[e] for t in it))[0]


if __name__ == "__main__":
    out = {}
    with Pool(8) as pool:
        for N, B in CASES:
            wl, _, _ = workload(N, B)
            ref = oracle.mpc_solve(N, K, wl.inputs, y0=1.0)
            x = np.stack(pool.map(one, [(N, B, e) for e in range(B)]))
            out[f"N{N}_B{B}"] = rel_err_rows(x, ref[0])
            print(N, B, f"max {out[f'N{N}_B{B}'].max():.1e}", flush=True)
    np.savez_compressed(os.path.join(HERE, "dense_floor_ragged.npz"), **out)
