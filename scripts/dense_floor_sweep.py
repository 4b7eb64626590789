"""CPU: the dense-LU restatement (oracle/pdipm_dense.py) against the C oracle over the same envs
scripts/parity_sweep.py uses: the FP64 spread two exact eliminations of the same KKT show, i.e. the
floor under any GPU-vs-oracle comparison. python scripts/dense_floor_sweep.py N GAIT K [SEEDS] [B]"""
import os
import sys
from multiprocessing import Pool

os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from biped_pympc_amd.utils.synthetic import make_workload, solver_init  # noqa: E402
from oracle import oracle  # noqa: E402
from oracle.pdipm_dense import pdipm_dense  # noqa: E402
from tests._util import rel_err_rows  # noqa: E402

N, gait, K = int(sys.argv[1]), bool(int(sys.argv[2])), int(sys.argv[3])
SEEDS = [int(s) for s in sys.argv[4].split(",")] if len(sys.argv) > 4 else [100, 101, 102, 103]
B = int(sys.argv[5]) if len(sys.argv) > 5 else 128


def one(args):
    seed, e = args
    wl = make_workload(B, N, seed=seed, random_gait=gait)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    it = solver_init(d, N)
    return pdipm_dense(N, K, H[e], G[e], A[e], f[e], d[e], b[e], *(t[e] for t in it))


if __name__ == "__main__":
    errs = []
    with Pool(8) as pool:
        for seed in SEEDS:
            wl = make_workload(B, N, seed=seed, random_gait=gait)
            H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
            it = solver_init(d, N)
            ref = oracle.pdipm(N, K, [H, G, A, f, d, b, *it])
            den = pool.map(one, [(seed, e) for e in range(B)])
            den = [np.stack(v) for v in zip(*den)]
            e = [rel_err_rows(den[k], ref[k]) for k in range(4)]
            e.append(rel_err_rows(den[0][:, 12 * N:12 * N + 12], ref[0][:, 12 * N:12 * N + 12]))
            errs.append(np.stack(e, 1))
    E = np.concatenate(errs)
    w = E[:, :4].max(1)
    print(f"dense-vs-oracle N={N} gait={int(gait)} K={K:2d} | x {E[:,0].max():.1e} s {E[:,1].max():.1e} "
          f"z {E[:,2].max():.1e} y {E[:,3].max():.1e} u0 {E[:,4].max():.1e} | >1e-8 {(w>1e-8).sum()} "
          f">1e-6 {(w>1e-6).sum()} >1e-5 {(w>1e-5).sum()} of {len(w)}", flush=True)
