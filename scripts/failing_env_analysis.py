"""Where a failing campaign env's HIP result sits among the three CPU restatements (CPU host; diagnostics).

    python scripts/failing_env_analysis.py FLOOR_REPORT.json ROWS.npz [POLICY ...]

FLOOR_REPORT: a scripts/parity_floor.py report (its failing envs, per policy); ROWS: the HIP rows of those
envs, from a scripts/parity_fuzz.py replay with FUZZ_SEEDS=<the failing seeds> FUZZ_ROWS=1 (same build).
Per failing env and output (x, s, z, y, u0): the HIP result's relative distance to the checker (exact
minimum-degree LDL^T), to the AMD-ordered LDL^T (the reference's ca.ldl order) and to dense LU, beside the
restatements' own spread -- whether the GPU is off all three, or sits among them and only the checker is
far from it.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    rep = json.load(open(sys.argv[1]))
    rows = np.load(sys.argv[2])
    pols = sys.argv[3:] or ["adaptive", "strict"]
    os.environ["FUZZ_CCS"] = "1" if rep["ccs"] else "0"
    import parity_fuzz as pf
    from oracle import oracle
    from oracle.pdipm_dense import pdipm_dense
    from tests._util import rel_err_rows
    params = pf.replay_all(max(c["seed"] for p in pols for c in rep["policies"][p]["failed"]))
    names = ["x", "s", "z", "y", "u0"]
    summary = []
    for p in pols:
        for c in rep["policies"][p]["failed"]:
            seed = c["seed"]
            N, K, B, entry, path, kw, y0, extra = params[seed]
            _, ins = pf.case_inputs(seed, N, K, B, entry, kw, y0, extra)
            u = slice(12 * N, 12 * N + 12)
            for f in c["fails"]:
                e = f["env"]
                key = f"{p}/{seed}/{e}"
                if f"{key}/x" not in rows.files:
                    print(f"{key}: no HIP rows in {sys.argv[2]}")
                    continue
                hip = [rows[f"{key}/{v}"][None] for v in "xszy"]
                one = [np.asarray(a)[e:e + 1] for a in ins]
                md = oracle.pdipm(N, K, one, nthreads=1)
                am = oracle.pdipm(N, K, one, nthreads=1, order="amd")
                dn = [np.asarray(v)[None] for v in pdipm_dense(N, K, *[a[0] for a in one])[:4]]

                def d(a, b):
                    return [float(rel_err_rows(a[k], b[k]).max()) for k in range(4)] + \
                           [float(rel_err_rows(a[0][:, u], b[0][:, u]).max())]
                g_md, g_am, g_dn = d(hip, md), d(hip, am), d(hip, dn)
                spread = [max(a, b, c_) for a, b, c_ in zip(d(am, md), d(dn, md), d(dn, am))]
                k = int(np.argmax([g / max(s, 1e-300) for g, s in zip(g_md, spread)]))
                near = min(g_md[k], g_am[k], g_dn[k])
                summary.append(near / max(spread[k], 1e-300))
                print(f"{p:9s} seed {seed} N{N:2d} K{K:2d} {entry:5s} {path:7s} env {e:3d} [{names[k]}] "
                      f"GPU-MD {g_md[k]:.1e} GPU-AMD {g_am[k]:.1e} GPU-LU {g_dn[k]:.1e} | spread {spread[k]:.1e} "
                      f"| nearest / spread {near / max(spread[k], 1e-300):.1f}")
    if summary:
        s = np.array(summary)
        print(f"{len(s)} envs: nearest restatement within the spread for {int((s <= 1).sum())}, within 4x for "
              f"{int((s <= 4).sum())}; median nearest / spread {np.median(s):.2f}, max {s.max():.1f}")


if __name__ == "__main__":
    main()
