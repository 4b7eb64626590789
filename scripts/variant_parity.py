"""Diagnostic: build compile-time variants of libsrbd_mpc.so into /tmp and compare their parity
with the oracle (run on the GPU box). Usage: python scripts/variant_parity.py NAME=-DFLAG ..."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
variants = [a.split("=", 1) for a in sys.argv[1:]] or [["base", ""]]
for name, flags in variants:
    out = f"/tmp/libsrbd_{name}.so"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    *[f for f in flags.split(",") if f], "-o", out,
                    os.path.join(ROOT, "biped_pympc_amd/csrc/srbd_mpc.hip")], check=True)
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
        e = [rel_err_rows(o[k], r[k]).max() for k in range(4)]
        u = rel_err_rows(o[0][:, 12*N:12*N+12], r[0][:, 12*N:12*N+12]).max()
        row.append(f"K{K}: x {e[0]:.1e} z {e[2]:.1e} y {e[3]:.1e} u0 {u:.1e}")
    print(f"  N={N} gait={gait} | " + " | ".join(row), flush=True)
''' % ROOT
for name, _ in variants:
    print(name, flush=True)
    env = dict(os.environ, SRBD_LIB=f"/tmp/libsrbd_{name}.so")
    subprocess.run([sys.executable, "-c", code], env=env, check=True)
