"""GPU box: solver parity vs the oracle per library variant (SRBD_LIB=path), several seeds.

    python scripts/parity_sweep.py NAME=LIB [NAME=LIB ...]      (LIB empty: the product library)

For each variant and (N, gait, K) prints, over SEEDS x B envs, the worst per-env relative error of
x, s, z, y, the first-stage input u0, and how many envs exceed 1e-8 / 1e-6 / 1e-5 in any of x/s/z/y.
Diagnostic only (the tests pin the product library)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
code = r'''
import sys, numpy as np, torch
sys.path.insert(0, %r)
from biped_pympc_amd import solver
from biped_pympc_amd.utils.synthetic import make_workload, solver_init
from oracle import oracle
from tests._util import rel_err_rows
def cuda(a): return [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in a]
B, SEEDS = 128, (100, 101, 102, 103)
for N in (10, 20):
    for gait in (False, True):
        for K in (1, 10, 20):
            errs = []
            for seed in SEEDS:
                wl = make_workload(B, N, seed=seed, random_gait=gait)
                H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
                it = solver_init(d, N)
                r = oracle.pdipm(N, K, [H, G, A, f, d, b, *it])
                o = solver.pdipm(cuda([H, G, A, f, d, b]), cuda(list(it)), N, K)
                torch.cuda.synchronize()
                o = [t.cpu().numpy() for t in o]
                e = [rel_err_rows(o[k], r[k]) for k in range(4)]
                e.append(rel_err_rows(o[0][:, 12*N:12*N+12], r[0][:, 12*N:12*N+12]))
                errs.append(np.stack(e, 1))
            E = np.concatenate(errs)
            w = E[:, :4].max(1)
            print(f"  N={N} gait={int(gait)} K={K:2d} | x {E[:,0].max():.1e} s {E[:,1].max():.1e} z {E[:,2].max():.1e} "
                  f"y {E[:,3].max():.1e} u0 {E[:,4].max():.1e} | >1e-8 {(w>1e-8).sum()} >1e-6 {(w>1e-6).sum()} "
                  f">1e-5 {(w>1e-5).sum()} of {len(w)}", flush=True)
''' % ROOT
for v in sys.argv[1:]:
    name, lib = v.split("=", 1)
    env = dict(os.environ, SRBD_LIB=lib) if lib else dict(os.environ)
    print(name, flush=True)
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=600)
