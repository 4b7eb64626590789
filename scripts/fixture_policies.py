"""The fuzz-regression fixture (tests/golden/fuzz_regressions.npz) under refinement policies (GPU box).

    python scripts/fixture_policies.py POLICY ...     (names of scripts/parity_fuzz.py POLICIES)

Per policy and fixture env: the errors against the stored oracle outputs over the test's own bounds
(tests/test_gpu_parity.py::test_fuzz_regressions: per output max(K tolerance, 4x floor); u0 max(1e-6, 4x
floor)); one JSON line per policy with the envs over their bound.
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from biped_pympc_amd import _native, solver  # noqa: E402
from parity_fuzz import policy_ctx, tol_for  # noqa: E402
from tests._util import rel_err_rows  # noqa: E402


def main():
    z = np.load(os.path.join(ROOT, "tests", "golden", "fuzz_regressions.npz"))
    keys = sorted({k.split("_")[0] for k in z.files})
    paths = {v: k for k, v in _native.SOLVER_PATHS.items()}
    for pol in sys.argv[1:]:
        over, worst = [], 0.0
        for key in keys:
            N, K, seed, env, path = (int(v) for v in z[f"{key}_NK"])
            ins = [torch.from_numpy(np.ascontiguousarray(z[f"{key}_in{j}"][None])).cuda() for j in range(10)]
            with policy_ctx(pol), _native.solver_path(paths[path]):
                out = solver.pdipm(ins[:6], ins[6:], N, K)
                torch.cuda.synchronize()
            fl = z[f"{key}_floor"]
            r = []
            for j in range(4):
                e = rel_err_rows(out[j].cpu().numpy(), z[f"{key}_ref{j}"][None])[0]
                r.append(e / max(tol_for(K), 4.0 * fl[j]))
            u = slice(12 * N, 12 * N + 12)
            eu = rel_err_rows(out[0].cpu().numpy()[:, u], z[f"{key}_ref0"][None, u])[0]
            r.append(eu / max(1e-6, 4.0 * fl[4]))
            worst = max(worst, max(r))
            if max(r) > 1.0:
                over.append({"key": key, "seed": seed, "env": env, "N": N, "K": K,
                             "over_bound": [round(float(v), 3) for v in r]})
        print(json.dumps({"policy": pol, "envs": len(keys), "over": over, "worst_over_bound": round(float(worst), 3)}),
              flush=True)


if __name__ == "__main__":
    main()
