"""Distance of the GPU and of the three FP64 restatements from an 80-bit extended-precision solve (CPU host;
diagnostics).

    python scripts/extended_precision_check.py FLOOR_REPORT.json ROWS.npz [POLICY]

The floor (scripts/parity_floor.py) is the spread of three FP64 restatements; an env beyond 4x it is "off
all three" (scripts/failing_env_analysis.py). This asks the next question: is the GPU further from the exact
answer than the restatements are, or are all four equally far and the GPU only far in another direction?
The exact answer is approximated by the dense restatement (oracle/pdipm_dense.py: the reference's KKT with
its BETA / DELTA regularisation, LU with partial pivoting) run in numpy's long double (64-bit mantissa,
2^-64 unit roundoff) with its own elimination -- the same algorithm, 2048x the precision.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

LD = np.longdouble
BETA = LD(1) / LD(10 ** 8)
DELTA = BETA


def _lu_solve(K, r):
    """Gaussian elimination with partial pivoting in long double (K small: N = 1..4)."""
    A = np.concatenate([K, r[:, None]], axis=1).astype(LD)
    n = A.shape[0]
    for c in range(n):
        p = c + int(np.argmax(np.abs(A[c:, c])))
        if p != c:
            A[[c, p]] = A[[p, c]]
        A[c + 1:, c:] -= np.outer(A[c + 1:, c] / A[c, c], A[c, c:])
    x = np.zeros(n, LD)
    for i in range(n - 1, -1, -1):
        x[i] = (A[i, n] - A[i, i + 1:n] @ x[i + 1:]) / A[i, i]
    return x


def _step(v, dv):
    c = dv < 0
    with np.errstate(divide="ignore", invalid="ignore"):
        a = -v / dv
    cand = np.where(c, a, LD(0)) + np.where(~c, LD(1), LD(0))
    return max(min(LD(1), LD(0.99) * np.fmin.reduce(cand)), LD(1e-12))


def pdipm_ld(N, n_iter, Hv, Gv, Av, f, h, b, x, s, z, y):
    """oracle/pdipm_dense.py's iteration (reference sparse_pdipm_solver.py:357-534) in long double."""
    from biped_pympc_amd import layout
    nz, m, p = 24 * N, 16 * N, 14 * N
    H = layout.to_dense(Hv, *layout.ccs_H(N), (nz, nz)).astype(LD)
    G = layout.to_dense(Gv, *layout.ccs_G(N), (m, nz)).astype(LD)
    A = layout.to_dense(Av, *layout.ccs_A(N), (p, nz)).astype(LD)
    f, h, b, x, s, z, y = (np.asarray(v, np.float64).astype(LD) for v in (f, h, b, x, s, z, y))
    n = nz + 2 * m + p
    for _ in range(n_iter):
        rx = H @ x + f + G.T @ z + A.T @ y
        re = A @ x - b
        rs = G @ x + s - h
        mu = s @ z / m
        sinv = LD(1) / s
        K = np.zeros((n, n), LD)
        K[:nz, :nz] = H + BETA * np.eye(nz, dtype=LD)
        K[:nz, nz + m:nz + 2 * m] = G.T
        K[:nz, nz + 2 * m:] = A.T
        K[nz:nz + m, nz:nz + m] = np.diag(sinv * z + DELTA)
        K[nz:nz + m, nz + m:nz + 2 * m] = np.eye(m, dtype=LD)
        K[nz + m:nz + 2 * m, :nz] = G
        K[nz + m:nz + 2 * m, nz:nz + m] = np.eye(m, dtype=LD)
        K[nz + m:nz + 2 * m, nz + m:nz + 2 * m] = -DELTA * np.eye(m, dtype=LD)
        K[nz + 2 * m:, :nz] = A
        K[nz + 2 * m:, nz + 2 * m:] = -DELTA * np.eye(p, dtype=LD)
        rhs = np.concatenate([-rx, -(sinv * (s * z)), -rs, -re])
        sa = _lu_solve(K, rhs)
        dsa, dza = sa[nz:nz + m], sa[nz + m:nz + 2 * m]
        ap, ad = _step(s, dsa), _step(z, dza)
        mu_aff = (s + ap * dsa) @ (z + ad * dza) / m
        sigma = (mu_aff / mu) ** 3
        rc = s * z + dsa * dza - sigma * mu
        rhs_c = np.concatenate([np.zeros(nz, LD), -(sinv * rc), np.zeros(m, LD), np.zeros(p, LD)])
        d = sa + _lu_solve(K, rhs_c)
        dx, ds, dz, dy = d[:nz], d[nz:nz + m], d[nz + m:nz + 2 * m], d[nz + 2 * m:]
        apc, adc = _step(s, ds), _step(z, dz)
        x = x + apc * dx
        s = np.fmax(s + apc * ds, LD(1e-8))
        z = np.fmax(z + adc * dz, LD(1e-8))
        y = y + adc * dy
    return [v.astype(np.float64)[None] for v in (x, s, z, y)], [v[None] for v in (x, s, z, y)]


def main():
    rep = json.load(open(sys.argv[1]))
    rows = np.load(sys.argv[2])
    pols = sys.argv[3:] or ["adaptive"]
    os.environ["FUZZ_CCS"] = "1" if rep["ccs"] else "0"
    import parity_fuzz as pf
    from oracle import oracle
    from oracle.pdipm_dense import pdipm_dense

    def rel(a, b):  # norm-wise relative distance of a to the long-double b, per output (x, s, z, y, u0)
        out = []
        for k in range(4):
            bb = b[k].astype(LD)
            out.append(float(np.abs(np.asarray(a[k], np.float64).astype(LD) - bb).max() / np.abs(bb).max()))
        bb = b[0][:, u].astype(LD)
        out.append(float(np.abs(np.asarray(a[0], np.float64)[:, u].astype(LD) - bb).max() / np.abs(bb).max()))
        return out

    names = ["x", "s", "z", "y", "u0"]
    params = pf.replay_all(max(c["seed"] for p in pols for c in rep["policies"][p]["failed"]))
    ratios = []
    for p in pols:
        for c in rep["policies"][p]["failed"]:
            seed = c["seed"]
            N, K, B, entry, path, kw, y0, extra = params[seed]
            if N > 4:
                continue
            _, ins = pf.case_inputs(seed, N, K, B, entry, kw, y0, extra)
            u = slice(12 * N, 12 * N + 12)
            for f in c["fails"]:
                e = f["env"]
                key = f"{p}/{seed}/{e}"
                if f"{key}/x" not in rows.files:
                    continue
                hip = [rows[f"{key}/{v}"][None] for v in "xszy"]
                one = [np.asarray(a)[e:e + 1] for a in ins]
                _, ex = pdipm_ld(N, K, *[a[0] for a in one])
                md = oracle.pdipm(N, K, one, nthreads=1)
                am = oracle.pdipm(N, K, one, nthreads=1, order="amd")
                dn = [np.asarray(v)[None] for v in pdipm_dense(N, K, *[a[0] for a in one])[:4]]
                g, r = rel(hip, ex), [rel(v, ex) for v in (md, am, dn)]
                k = int(np.argmax([g[j] / max(max(q[j] for q in r), 1e-300) for j in range(5)]))
                worst = max(q[k] for q in r)
                ratios.append(g[k] / max(worst, 1e-300))
                print(f"{p:9s} seed {seed} N{N} K{K:2d} {entry:5s} {path:7s} env {e:3d} [{names[k]}] "
                      f"GPU-exact {g[k]:.1e} | MD-exact {r[0][k]:.1e} AMD-exact {r[1][k]:.1e} "
                      f"LU-exact {r[2][k]:.1e} | GPU / worst restatement {g[k] / max(worst, 1e-300):.1f}",
                      flush=True)
    if ratios:
        s = np.array(ratios)
        print(f"{len(s)} envs: GPU further from the long-double answer than the furthest FP64 restatement in "
              f"{int((s > 1).sum())}; median ratio {np.median(s):.2f}, max {s.max():.1f}")


if __name__ == "__main__":
    main()
