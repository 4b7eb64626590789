"""GPU box: parity + fused-step time per library variant (SRBD_LIB=path), one subprocess each."""
import json, os, subprocess, sys
ROOT = "/root/repo"
variants = sys.argv[1:]
code = r'''
import sys, numpy as np, torch
sys.path.insert(0, %r)
from biped_pympc_amd import solver
from biped_pympc_amd.utils.synthetic import make_workload, solver_init
from oracle import oracle
from tests._util import rel_err_rows
def cuda(a): return [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in a]
for N, gait in ((10, False), (10, True), (20, True)):
    wl = make_workload(64, N, seed=100, random_gait=gait)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    it = solver_init(d, N)
    row = []
    for K in (1, 5, 10, 20):
        r = oracle.pdipm(N, K, [H, G, A, f, d, b, *it])
        o = solver.pdipm(cuda([H, G, A, f, d, b]), cuda(list(it)), N, K)
        torch.cuda.synchronize()
        o = [t.cpu().numpy() for t in o]
        e = max(rel_err_rows(o[k], r[k]).max() for k in range(4))
        row.append(f"K{K} {e:.1e}")
    print(f"  N={N} gait={gait} | " + " ".join(row), flush=True)
''' % ROOT
for v in variants:
    name, lib = v.split("=", 1)
    env = dict(os.environ, SRBD_LIB=lib) if lib else dict(os.environ)
    print(name, flush=True)
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
    for N in (10, 20):
        out = subprocess.run([sys.executable, "bench.py", "--steps", "50", "--warmup", "5", "--no-cpu-baseline",
                              "--horizon", str(N)], env=env, check=True, timeout=300, capture_output=True, text=True).stdout
        d = json.loads(out.strip().splitlines()[-1])
        print(f"  N={N} fused step {d['kernels_ms']['mpc_step_fused']:.4f} ms", flush=True)
