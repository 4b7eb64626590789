"""Dense numpy restatement of ``sparse_pdipm_multiple_iterations`` (TEST INFRASTRUCTURE ONLY).

A second, independent restatement of reference ``biped_pympc/casadi/sparse_pdipm_solver.py:357-534``
used only to cross-validate the C oracle (``srbd_oracle.c``): it assembles the same 70N x 70N KKT
densely and solves it with LAPACK LU (partial pivoting) instead of a sparse LDL^T, so agreement
between the two pins the algebra rather than one factorisation's rounding. Small N / few envs only.
"""
from __future__ import annotations

import numpy as np

from biped_pympc_amd import layout

BETA = 1e-8
DELTA = 1e-8


def _if_else_step(v, dv):
    c = dv < 0
    with np.errstate(divide="ignore", invalid="ignore"):
        a = -v / dv
    cand = np.where(c, a, 0.0) + np.where(~c, 1.0, 0.0)
    return max(min(1.0, 0.99 * np.fmin.reduce(cand)), 1e-12)


def pdipm_dense(N: int, n_iter: int, Hv, Gv, Av, f, h, b, x, s, z, y, factor_once: bool = False):
    """factor_once: one LU (scipy lu_factor) per iteration for both solves -- the same restatement at half
    the cost, for the parity campaign's per-env floors (scripts/parity_floor.py)."""
    nz, m, p = 24 * N, 16 * N, 14 * N
    H = layout.to_dense(Hv, *layout.ccs_H(N), (nz, nz))
    G = layout.to_dense(Gv, *layout.ccs_G(N), (m, nz))
    A = layout.to_dense(Av, *layout.ccs_A(N), (p, nz))
    x, s, z, y = (np.array(v, np.float64) for v in (x, s, z, y))
    n = nz + 2 * m + p
    res = np.zeros(4)
    mu_new = 0.0
    for _ in range(n_iter):
        rx = H @ x + f + G.T @ z + A.T @ y
        re = A @ x - b
        rs = G @ x + s - h
        mu = s @ z / m
        sinv = 1.0 / s
        K = np.zeros((n, n))
        K[:nz, :nz] = H + BETA * np.eye(nz)
        K[:nz, nz + m:nz + 2 * m] = G.T
        K[:nz, nz + 2 * m:] = A.T
        K[nz:nz + m, nz:nz + m] = np.diag(sinv * z + DELTA)
        K[nz:nz + m, nz + m:nz + 2 * m] = np.eye(m)
        K[nz + m:nz + 2 * m, :nz] = G
        K[nz + m:nz + 2 * m, nz:nz + m] = np.eye(m)
        K[nz + m:nz + 2 * m, nz + m:nz + 2 * m] = -DELTA * np.eye(m)
        K[nz + 2 * m:, :nz] = A
        K[nz + 2 * m:, nz + 2 * m:] = -DELTA * np.eye(p)
        rhs = np.concatenate([-rx, -(sinv * (s * z)), -rs, -re])
        if factor_once:
            from scipy.linalg import lu_factor, lu_solve
            lu = lu_factor(K, check_finite=False)
            solve = lambda r: lu_solve(lu, r, check_finite=False)  # noqa: E731
        else:
            solve = lambda r: np.linalg.solve(K, r)  # noqa: E731
        sa = solve(rhs)
        dsa, dza = sa[nz:nz + m], sa[nz + m:nz + 2 * m]
        ap, ad = _if_else_step(s, dsa), _if_else_step(z, dza)
        mu_aff = (s + ap * dsa) @ (z + ad * dza) / m
        sigma = (mu_aff / mu) ** 3
        rc = s * z + dsa * dza - sigma * mu
        rhs_c = np.concatenate([np.zeros(nz), -(sinv * rc), np.zeros(m), np.zeros(p)])
        d = sa + solve(rhs_c)
        dx, ds, dz, dy = d[:nz], d[nz:nz + m], d[nz + m:nz + 2 * m], d[nz + 2 * m:]
        apc, adc = _if_else_step(s, ds), _if_else_step(z, dz)
        x = x + apc * dx
        s = np.fmax(s + apc * ds, 1e-8)
        z = np.fmax(z + adc * dz, 1e-8)
        y = y + adc * dy
        mu_new = s @ z / m
        res = np.array([np.linalg.norm(rx), np.linalg.norm(rs), np.linalg.norm(re), mu_new])
    return x, s, z, y, res, np.array([mu_new])
