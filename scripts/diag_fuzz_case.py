"""Diagnose one env of a scripts/parity_fuzz.py case on the GPU: the iterate trajectory of the HIP path
(auto and lds) against the oracle, iteration by iteration, and one-iteration errors from the oracle's own
iterate (is an iteration inaccurate, or is an early difference amplified?).

    python scripts/diag_fuzz_case.py SEED ENV [SEED ENV ...]     (FUZZ_CCS=1 for the campaign with the _ccs entry)
"""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
import parity_fuzz as pf  # noqa: E402
from biped_pympc_amd import _native, solver  # noqa: E402
from oracle import oracle  # noqa: E402
from tests._util import rel_err_rows  # noqa: E402


def cu(a):
    return [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in a]


def main():
    args = sys.argv[1:]
    for seed, env in zip(args[::2], args[1::2]):
        seed, env = int(seed), int(env)
        N, K, B, entry, path, kw, y0, extra = pf.replay(seed)
        _, ins = pf.case_inputs(seed, N, K, B, entry, kw, y0, extra)
        H, G, A, f, d, b = ins[:6]
        it = ins[6:]
        qp = [a[env:env + 1] for a in (H, G, A, f, d, b)]
        it = [a[env:env + 1] for a in it]
        print(f"# seed {seed} env {env}: N={N} K={K} entry={entry} path={path} {extra} y0={y0} kw={ {k: v for k, v in kw.items() if k != 'contact_override'} }")
        print("#  k | x s z y err vs oracle (trajectory): auto | lds | general | auto 1-iter from the oracle's iterate k-1 | mu_k, min s, max z/s, max|z|")
        cur = it
        for k in range(1, K + 1):
            ref = oracle.pdipm(N, k, qp + it)
            row = []
            for p in ("auto", "lds", "general"):
                with _native.solver_path(p), _native.refinement(pf.REFINE):
                    g = solver.pdipm(cu(qp), cu(it), N, k)
                torch.cuda.synchronize()
                row.append([float(rel_err_rows(g[j].cpu().numpy(), ref[j]).max()) for j in range(4)])
            with _native.solver_path("auto"), _native.refinement(pf.REFINE):
                g1 = solver.pdipm(cu(qp), cu(cur), N, 1)
            torch.cuda.synchronize()
            r1 = oracle.pdipm(N, 1, qp + cur)
            one = [float(rel_err_rows(g1[j].cpu().numpy(), r1[j]).max()) for j in range(4)]
            mu = float(ref[5][0][0]) if ref[5].size else float("nan")
            print(f"{k:4d} | " + " | ".join(" ".join(f"{e:.1e}" for e in r) for r in row) +
                  " | " + " ".join(f"{e:.1e}" for e in one) +
                  f" | {mu:.2e} {float(cur[1].min()):.1e} {float((cur[2] / cur[1]).max()):.1e} {float(np.abs(cur[2]).max()):.1e}")
            cur = [r.copy() for r in ref[:4]]


if __name__ == "__main__":
    main()
