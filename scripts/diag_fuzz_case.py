"""Diagnose one env of a scripts/parity_fuzz.py case on the GPU: the iterate trajectory of the HIP path
(auto and lds) against the oracle, iteration by iteration, and one-iteration errors from the oracle's own
iterate (is an iteration inaccurate, or is an early difference amplified?).

    python scripts/diag_fuzz_case.py SEED ENV [SEED ENV ...]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.abspath(__file__)))
import parity_fuzz as pf  # noqa: E402
from biped_pympc_amd import _native, solver  # noqa: E402
from biped_pympc_amd.utils.synthetic import make_workload, solver_init  # noqa: E402
from oracle import oracle  # noqa: E402
from tests._util import rel_err_rows  # noqa: E402


def replay(seed_want):
    rng = np.random.default_rng(20261018)
    seed = 50000
    while True:
        N, K, B, entry, path, kw, y0 = pf.draw(rng)
        K0 = int(rng.integers(1, 11)) if entry == "warm" else 0
        if seed == seed_want:
            return N, K, B, entry, path, kw, y0, K0
        seed += 1


def cu(a):
    return [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in a]


def main():
    args = sys.argv[1:]
    for seed, env in zip(args[::2], args[1::2]):
        seed, env = int(seed), int(env)
        N, K, B, entry, path, kw, y0, K0 = replay(seed)
        wl = make_workload(B, N, seed=seed, **kw)
        H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
        it = list(solver_init(d, N, y0))
        if entry == "warm":
            it = oracle.pdipm(N, K0, [H, G, A, f, d, b, *it])[:4]
        qp = [a[env:env + 1] for a in (H, G, A, f, d, b)]
        it = [a[env:env + 1] for a in it]
        print(f"# seed {seed} env {env}: N={N} K={K} entry={entry} K0={K0} y0={y0} kw={ {k: v for k, v in kw.items() if k != 'contact_override'} }")
        print("#  k | auto: x s z y err vs oracle (trajectory)      | lds: same          | auto 1-iter from oracle iterate k-1 | mu_k, min s")
        cur = it
        for k in range(1, K + 1):
            ref = oracle.pdipm(N, k, qp + it)
            row = []
            for p in ("auto", "lds"):
                with _native.solver_path(p):
                    g = solver.pdipm(cu(qp), cu(it), N, k)
                torch.cuda.synchronize()
                row.append([float(rel_err_rows(g[j].cpu().numpy(), ref[j]).max()) for j in range(4)])
            with _native.solver_path("auto"):
                g1 = solver.pdipm(cu(qp), cu(cur), N, 1)
            torch.cuda.synchronize()
            r1 = oracle.pdipm(N, 1, qp + cur)
            one = [float(rel_err_rows(g1[j].cpu().numpy(), r1[j]).max()) for j in range(4)]
            mu = float(ref[5][0][0]) if ref[5].size else float("nan")
            print(f"{k:4d} | " + " ".join(f"{e:.1e}" for e in row[0]) + " | " + " ".join(f"{e:.1e}" for e in row[1]) +
                  " | " + " ".join(f"{e:.1e}" for e in one) + f" | {mu:.2e} {float(ref[1].min()):.1e}")
            cur = [r.copy() for r in ref[:4]]


if __name__ == "__main__":
    main()
