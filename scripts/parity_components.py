"""GPU diag: which components of x carry the K=1 error, per solver path."""
import sys, numpy as np, torch
sys.path.insert(0, "/root/repo")
from biped_pympc_amd import solver, _native
from biped_pympc_amd.utils.synthetic import make_workload, solver_init
from oracle import oracle
from oracle.pdipm_dense import pdipm_dense


def cuda(a):
    return [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in a]


names = ["x", "s", "z", "y"]
for N in (10, 20):
    wl = make_workload(64, N, seed=101, random_gait=False)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    it = solver_init(d, N)
    for K in (1, 2, 5, 10):
        ref = oracle.pdipm(N, K, [H, G, A, f, d, b, *it])
        den = [np.stack(v) for v in zip(*[pdipm_dense(N, K, H[e], G[e], A[e], f[e], d[e], b[e], *(t[e] for t in it)) for e in range(8)])]
        for path in ("auto", "general", "lds"):
            with _native.solver_path(path):
                o = solver.pdipm(cuda([H, G, A, f, d, b]), cuda(list(it)), N, K)
                torch.cuda.synchronize()
            o = [t.cpu().numpy() for t in o]
            msg = []
            for k in range(4):
                err = np.abs(o[k] - ref[k])
                sc = np.abs(ref[k]).max(axis=1, keepdims=True)
                rel = (err / sc)
                e = int(rel.max(axis=1).argmax())
                idx = int(rel[e].argmax())
                msg.append(f"{names[k]} {rel.max():.1e}@{idx}")
            # where is x error: states vs inputs per component
            relx = np.abs(o[0] - ref[0]) / np.abs(ref[0]).max(axis=1, keepdims=True)
            ux = relx[:, 12 * N:].reshape(64, N, 12).max(axis=(0, 1))
            xx = relx[:, :12 * N].reshape(64, N, 12).max(axis=(0, 1))
            print(f"N={N} K={K} {path:8s} " + " ".join(msg), flush=True)
            print("   u comps " + " ".join(f"{v:.0e}" for v in ux), flush=True)
            print("   x comps " + " ".join(f"{v:.0e}" for v in xx), flush=True)
        dd = [np.abs(den[k] - ref[k][:8]).max(axis=1) / np.abs(ref[k][:8]).max(axis=1) for k in range(4)]
        print(f"N={N} K={K} dense-vs-oracle " + " ".join(f"{names[k]} {dd[k].max():.1e}" for k in range(4)), flush=True)
