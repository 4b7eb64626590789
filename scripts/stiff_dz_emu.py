"""CPU emulation (numpy) of one Newton system at an iterate where the kernels' dz drifts (a parity-campaign
env, replayed): the dz the reduced elimination produces when the Phi solve is an explicit inverse (the
kernels' sweep) against an LU solve of Phi, each with one and two refinement steps of KKT rows 1 + 4, and
against the full KKT solved by LU with long-double refinement (the reference's answer). Tests the DESIGN
7b hypothesis that the explicit inverse loses the stiff direction G_i dx at rows with W = z / s ~ 1e7..1e8.

    FUZZ_CCS=1 python scripts/stiff_dz_emu.py SEED ENV K     (K: the iteration whose Newton system is emulated)
"""
import os
import sys

import numpy as np
import scipy.linalg as sl

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import parity_fuzz as pf  # noqa: E402
from biped_pympc_amd import layout  # noqa: E402
from oracle import oracle  # noqa: E402

BETA = DELTA = 1e-8


def sweep_inv(a):
    """The kernels' symmetric sweep inverse (scripts/dual_refine_emu.py sweep_inv)."""
    a = a.copy()
    for k in range(a.shape[0]):
        idk = 1.0 / a[k, k]
        col = a[:, k].copy()
        a2 = a - np.outer(col, col) * idk
        a2[k, :] = a[k, :] * idk; a2[:, k] = a[:, k] * idk; a2[k, k] = -idk
        a = a2
    return -a


def main(seed, env, K):
    N, Kc, B, entry, path, kw, y0, extra = pf.replay(seed)
    wl, ins = pf.case_inputs(seed, N, Kc, B, entry, kw, y0, extra)
    ins = [np.ascontiguousarray(a[env:env + 1]) for a in ins]
    it = ins[6:]
    if K > 1:
        it = oracle.pdipm(N, K - 1, ins)[:4]
    x, s, z, y = (a[0] for a in it)
    Hv, Gv, Av, f, h, b = (a[0] for a in ins[:6])
    nz, m, p = 24 * N, 16 * N, 14 * N
    H = layout.to_dense(Hv, *layout.ccs_H(N), (nz, nz))
    G = layout.to_dense(Gv, *layout.ccs_G(N), (m, nz))
    A = layout.to_dense(Av, *layout.ccs_A(N), (p, nz))
    rx = H @ x + f + G.T @ z + A.T @ y; re = A @ x - b; rs = G @ x + s - h
    W = z / s + DELTA; Dd = 1 + DELTA * W; Lam = W / Dd
    r1, r2, r3, r4 = -rx, -(s * z) / s, -rs, -re   # the affine system, r2 in the s-scaled form
    Phi = H + BETA * np.eye(nz) + G.T @ (Lam[:, None] * G)
    r1t = r1 - G.T @ ((r2 - W * r3) / Dd)
    n = nz + 2 * m + p
    Kk = np.zeros((n, n))
    Kk[:nz, :nz] = H + BETA * np.eye(nz); Kk[:nz, nz + m:nz + 2 * m] = G.T; Kk[:nz, nz + 2 * m:] = A.T
    Kk[nz:nz + m, nz:nz + m] = np.diag(W); Kk[nz:nz + m, nz + m:nz + 2 * m] = np.eye(m)
    Kk[nz + m:nz + 2 * m, :nz] = G; Kk[nz + m:nz + 2 * m, nz:nz + m] = np.eye(m)
    Kk[nz + m:nz + 2 * m, nz + m:nz + 2 * m] = -DELTA * np.eye(m)
    Kk[nz + 2 * m:, :nz] = A; Kk[nz + 2 * m:, nz + 2 * m:] = -DELTA * np.eye(p)
    rhs = np.concatenate([r1, r2, r3, r4])
    lu = sl.lu_factor(Kk); sol = sl.lu_solve(lu, rhs)
    Kl, rl = Kk.astype(np.longdouble), rhs.astype(np.longdouble)
    for _ in range(4):
        sol = sol + sl.lu_solve(lu, (rl - Kl @ sol.astype(np.longdouble)).astype(np.float64))
    dz_ref = sol[nz + m:nz + 2 * m]
    PhiS = sweep_inv(Phi)
    S = A @ np.linalg.solve(Phi, A.T) + DELTA * np.eye(p)   # the dual Schur complement from an exact Phi solve
    S_sweep = A @ PhiS @ A.T + DELTA * np.eye(p)            # ... and from the sweep inverse (as the kernels)
    lus_exact, lus_sweep = sl.lu_factor(S), sl.lu_factor(S_sweep)

    def reduced(phis, steps, lus):
        g = A @ phis(r1t) - r4
        yy = sl.lu_solve(lus, g)
        dx = phis(r1t - A.T @ yy)
        for _ in range(steps):  # KKT rows 1 + 4 on the reduced system
            e1 = r1t - (Phi @ dx + A.T @ yy)
            e4 = r4 - (A @ dx - DELTA * yy)
            cy = sl.lu_solve(lus, A @ phis(e1) - e4)
            dx = dx + phis(e1 - A.T @ cy); yy = yy + cy
        gd = G @ dx
        return (r2 - W * r3) / Dd + Lam * gd

    sc = np.abs(dz_ref).max()
    hi = W > 1e6
    print(f"seed {seed} env {env} N={N} iteration {K}: max W {W.max():.1e}, rows with W > 1e6: {int(hi.sum())}, "
          f"cond Phi {np.linalg.cond(Phi):.1e}")
    lu_phi = sl.lu_factor(Phi)
    variants = (("explicit inverse, exact S", lambda v: PhiS @ v, lus_exact),
                ("LU solve of Phi, exact S", lambda v: sl.lu_solve(lu_phi, v), lus_exact),
                ("explicit inverse, sweep S", lambda v: PhiS @ v, lus_sweep),
                ("LU solve of Phi, sweep S", lambda v: sl.lu_solve(lu_phi, v), lus_sweep))
    for name, phis, lus in variants:
        for steps in (0, 1, 2):
            dz = reduced(phis, steps, lus)
            err = np.abs(dz - dz_ref) / sc
            print(f"  {name:30s} refinement steps {steps}: dz rel err max {err.max():.1e}, at W > 1e6 rows "
                  f"{err[hi].max() if hi.any() else 0:.1e}, elsewhere {err[~hi].max():.1e}")


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]))
