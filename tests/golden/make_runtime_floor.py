"""Generate tests/golden/dense_floor_runtime.npz (committed fixture; CPU, ~1 min on 8 cores).

For the runtime-horizon workloads of tests/test_gpu_parity.py::test_runtime_horizon_solver_matches_oracle
(N in {1, 2, 3, 5, 15, 16, 25, 32}, B = 48, randomized gait, seed 500 + N, GPU-caller init) at K = 1, 5, 10, 20:
the per-env relative error of x, s, z, y between the two independent CPU restatements of the
solver -- the C oracle (sparse LDL^T) and oracle/pdipm_dense.py (dense LU of the full KKT). That
spread is the FP64 floor of the comparison; the GPU test allows max(tol, 4 x floor) per env.
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

HORIZONS = (1, 2, 3, 5, 15, 16, 25, 32)
B = 48


def workload(N):
    wl = make_workload(B, N, seed=500 + N, random_gait=True)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    return [H, G, A, f, d, b], solver_init(d, N)


KS = (1, 5, 10, 20)


def one(args):
    N, e = args
    qp, it = workload(N)
    q = [a[e] for a in qp]
    cur, done, out = [t[e] for t in it], 0, []
    for K in KS:  # iterations compose: 1 + 4 + 5 + 10
        cur = pdipm_dense(N, K - done, *q, *cur)[:4]
        done = K
        out.append(cur)
    return out


if __name__ == "__main__":
    out = {}
    with Pool(8) as pool:
        for N in HORIZONS:
            qp, it = workload(N)
            dense = pool.map(one, [(N, e) for e in range(B)])
            for ki, K in enumerate(KS):
                ref = oracle.pdipm(N, K, qp + list(it))
                for k, v in enumerate("xszy"):
                    dv = np.stack([dense[e][ki][k] for e in range(B)])
                    out[f"N{N}_K{K}_{v}"] = rel_err_rows(dv, ref[k])
                print(N, K, " ".join(f"{v} {out[f'N{N}_K{K}_{v}'].max():.1e}" for v in "xszy"), flush=True)
    np.savez_compressed(os.path.join(HERE, "dense_floor_runtime.npz"), **out)
