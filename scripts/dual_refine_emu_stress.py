"""CPU emulation (numpy) of the solver kernels' dual-Schur elimination on one Newton system of a STRESS env
(tests/_stress.py) at iterations K (iterate from the dense restatement), against the full KKT solved by
LU with long-double refinement: direction errors of the unrefined reduced solve, of refinement from
KKT rows 1 + 4 only, and of refinement from all four rows (the kernel form: e1 on the foot columns,
e4 on the dynamics rows), and of the affine direction with and without it. Diagnostic for
pdipm_srbd_reg.hpp RegCtx::refine_rhs.
    python scripts/dual_refine_emu_stress.py CASE K1,K2,.. ENV      e.g. tilt_N10 17,18,19,20 11"""
import os, sys
import numpy as np, scipy.linalg as sl
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biped_pympc_amd import layout
from biped_pympc_amd.utils.synthetic import make_workload, solver_init
from oracle import oracle
from oracle.pdipm_dense import pdipm_dense
BETA = DELTA = 1e-8
from tests._stress import stress_workload
CASE = sys.argv[1]; KS = [int(k) for k in sys.argv[2].split(",")]; ENV = int(sys.argv[3])
E = 1

N, wl = stress_workload(CASE); wl.inputs = [a[ENV:ENV + 1] for a in wl.inputs]
Hv, fv, Av, bv, Gv, dv = oracle.qp_former(N, wl.inputs)
print("case", CASE, "env", ENV)
it0 = solver_init(dv, N)
nz, m, p = 24 * N, 16 * N, 14 * N
perm = np.concatenate([np.r_[12 * i:12 * i + 12, 12 * N + 2 * i, 12 * N + 2 * i + 1] for i in range(N)])
inv_perm = np.argsort(perm)

def sweep_inv(a):
    a = a.copy(); n = a.shape[0]
    for k in range(n):
        idk = 1.0 / a[k, k]
        col = a[:, k].copy()
        a2 = a - np.outer(col, col) * idk
        a2[k, :] = a[k, :] * idk; a2[:, k] = a[:, k] * idk; a2[k, k] = -idk
        a = a2
    return -a

def gj_rows(a):
    a = a.copy(); n = a.shape[0]; sc = np.ones(n)
    for k in range(n):
        pk = a[k].copy(); idk = 1.0 / pk[k]
        t = a[:, k] * idk; t[k] = 0.0
        a = a - np.outer(t, pk); a[:, k] = t; a[k, :] = pk; a[k, k] = -1.0; sc[k] = idk
    return -(a * sc[:, None])
def gj_mixed(a):
    r = gj_rows(a); return np.triu(r) + np.triu(r, 1).T

def block_solve(S, g, bs, inv):
    n = len(g) // bs
    B = lambda i, j: S[i * bs:(i + 1) * bs, j * bs:(j + 1) * bs]
    Dinv, w = [], []
    for i in range(n):
        D = B(i, i).copy(); q = g[i * bs:(i + 1) * bs].copy()
        if i:
            C = B(i, i - 1); D = D - C @ Dinv[-1] @ C.T; q = q - C @ w[-1]
        Di = inv(D); Dinv.append(Di); w.append(Di @ q)
    y = [None] * n; y[-1] = w[-1]
    for i in range(n - 2, -1, -1):
        y[i] = w[i] - Dinv[i] @ (B(i + 1, i).T @ y[i + 1])
    return np.concatenate(y)

res = {}
for K in KS:
    for e in range(E):
        H = layout.to_dense(Hv[e], *layout.ccs_H(N), (nz, nz))
        G = layout.to_dense(Gv[e], *layout.ccs_G(N), (m, nz))
        A = layout.to_dense(Av[e], *layout.ccs_A(N), (p, nz))
        f, h, b = fv[e], dv[e], bv[e]
        if K > 1:
            x, s, z, y, _, _ = pdipm_dense(N, K - 1, Hv[e], Gv[e], Av[e], f, h, b, *(t[e] for t in it0))
        else:
            x, s, z, y = (t[e].copy() for t in it0)
        rx = H @ x + f + G.T @ z + A.T @ y; re = A @ x - b; rs = G @ x + s - h
        W = z / s + DELTA; Dd = 1 + DELTA * W; Lam = W / Dd
        r1, r2, r3, r4 = -rx, -(1 / s * (s * z)), -rs, -re
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
        dense_x = sol[:nz].copy()
        Kl, rl = Kk.astype(np.longdouble), rhs.astype(np.longdouble)
        for _ in range(3):
            sol = sol + sl.lu_solve(lu, (rl - Kl @ sol.astype(np.longdouble)).astype(np.float64))
        xref = sol[:nz]
        out = {"dense_lu": dense_x}
        PhiS = sweep_inv(Phi)
        S = A @ PhiS @ A.T + DELTA * np.eye(p)
        Sp = S[np.ix_(perm, perm)]
        solveS = lambda v: block_solve(Sp, v[perm], 14, gj_mixed)[inv_perm]
        for name, phis in (("dual_sweepPhi", lambda v: PhiS @ v), ("dual_exactPhi", lambda v: np.linalg.solve(Phi, v))):
            g = A @ phis(r1t) - r4
            y0 = solveS(g)
            t = phis(r1t); dx0 = t - phis(A.T @ y0)
            out[name + "_unref"] = dx0
            rho = A @ dx0 - DELTA * y0 - r4
            c = solveS(rho)
            out[name] = dx0 - phis(A.T @ c)
            # two steps
            y1 = y0 + c; dx1 = out[name]
            rho = A @ dx1 - DELTA * y1 - r4
            out[name + "2"] = dx1 - phis(A.T @ solveS(rho))
        # full KKT refinement (rows 1, 4) with sweep Phi
        def full_solve(r1t_, r4_):
            g = A @ (PhiS @ r1t_) - r4_
            yy = solveS(g); return PhiS @ (r1t_ - A.T @ yy), yy
        dx0, y0 = full_solve(r1t, r4)
        e1 = r1t - (Phi @ dx0 + A.T @ y0)
        e4 = r4 - (A @ dx0 - DELTA * y0)
        cx, cy = full_solve(e1, e4)
        out["full_ref"] = dx0 + cx
        # refinement against ALL FOUR KKT rows, the reduced (dual-Schur) solver as the correction solver
        def solve_red(q1, q2, q3, q4, phis=lambda v: PhiS @ v):
            r1t_ = q1 - G.T @ ((q2 - W * q3) / Dd)
            g_ = A @ phis(r1t_) - q4
            yy = solveS(g_)
            dxx = phis(r1t_ - A.T @ yy)
            dzz = (q2 - W * q3) / Dd + Lam * (G @ dxx)
            dss = q3 - G @ dxx + DELTA * dzz
            return np.concatenate([dxx, dss, dzz, yy])
        d4 = solve_red(r1, r2, r3, r4)
        out["red4_unref"] = d4[:nz].copy()
        def solve_red_g(q1, q2, q3, q4, phis=lambda v: PhiS @ v):
            r1t_ = q1 - G.T @ ((q2 - W * q3) / Dd)
            g_ = A @ phis(r1t_) - q4
            yy = solveS(g_)
            dxx = phis(r1t_ - A.T @ yy)
            pr = q3 - G @ dxx
            dzz = (q2 - W * pr) / Dd
            dss = pr + DELTA * dzz
            return np.concatenate([dxx, dss, dzz, yy])
        full_true = sol
        foot = np.zeros(nz, bool)
        for i_ in range(N):
            for j_ in (0, 1, 2, 7, 3, 4, 5, 10):
                foot[12 * N + 12 * i_ + j_] = True
        # cheap correction without the dual chain solve: rows 1 (foot) - 3 only, c_y = 0
        def corr_nodual(dd, phis=lambda v: PhiS @ v):
            e = rhs - Kk @ dd
            q1, q2, q3 = np.where(foot, e[:nz], 0.0), e[nz:nz + m], e[nz + m:nz + 2 * m]
            qq = (q2 - W * q3) / Dd
            tc = phis(q1 - G.T @ qq)
            cz = qq + Lam * (G @ tc)
            cs = q3 - G @ tc + DELTA * cz
            return dd + np.concatenate([tc, cs, cz, np.zeros(p)])
        base = solve_red(r1, r2, r3, r4)
        for tag, dd in (("unref", base), ("nodual1", corr_nodual(base)), ("nodual2", corr_nodual(corr_nodual(base)))):
            rel = lambda a, b: np.abs(a - b).max() / np.abs(b).max()
            print(f"K={K} affine {tag}: dx {rel(dd[:nz], sol[:nz]):.1e} ds {rel(dd[nz:nz+m], sol[nz:nz+m]):.1e} dz {rel(dd[nz+m:nz+2*m], sol[nz+m:nz+2*m]):.1e}")
        dg = solve_red_g(r1, r2, r3, r4)
        sc_all = np.abs(full_true).max()
        for tag, dd in (("form_cancel", d4), ("form_grouped", dg)):
            print(f"K={K} {tag}: dx {np.abs(dd[:nz]-full_true[:nz]).max()/np.abs(full_true[:nz]).max():.1e} "
                  f"ds {np.abs(dd[nz:nz+m]-full_true[nz:nz+m]).max()/np.abs(full_true[nz:nz+m]).max():.1e} "
                  f"dz {np.abs(dd[nz+m:nz+2*m]-full_true[nz+m:nz+2*m]).max()/np.abs(full_true[nz+m:nz+2*m]).max():.1e}")
        ee = rhs - Kk @ dg
        for step in range(1, 3):
            dg = dg + solve_red_g(ee[:nz] if True else 0, ee[nz:nz + m], ee[nz + m:nz + 2 * m], ee[nz + 2 * m:])
            ee = rhs - Kk @ dg
        e1f = (rhs - Kk @ solve_red_g(r1, r2, r3, r4))
        # rows 1 + 4 only refinement on the grouped form
        dgg = solve_red_g(r1, r2, r3, r4)
        e = rhs - Kk @ dgg
        dgg = dgg + solve_red_g(e[:nz], np.zeros(m), np.zeros(m), e[nz + 2 * m:])
        print(f"K={K} grouped + rows1,4 ref: dx {np.abs(dgg[:nz]-full_true[:nz]).max()/np.abs(full_true[:nz]).max():.1e} dz {np.abs(dgg[nz+m:nz+2*m]-full_true[nz+m:nz+2*m]).max()/np.abs(full_true[nz+m:nz+2*m]).max():.1e}")
        for step in range(1, 4):
            e = (rl - Kl @ d4.astype(np.longdouble)).astype(np.float64)
            d4 = d4 + solve_red(e[:nz], e[nz:nz + m], e[nz + m:nz + 2 * m], e[nz + 2 * m:])
            out[f"red4_ref{step}"] = d4[:nz].copy()
        # FP64 residuals (what the GPU can do): rows 1-4 in double
        d4 = solve_red(r1, r2, r3, r4)
        for step in range(1, 3):
            e = rhs - Kk @ d4
            d4 = d4 + solve_red(e[:nz], e[nz:nz + m], e[nz + m:nz + 2 * m], e[nz + 2 * m:])
            out[f"red4_fp64_ref{step}"] = d4[:nz].copy()
        # FP64 residuals, e1 kept on the foot columns only and e4 on the dynamics rows only (kernel form)
        foot = np.zeros(nz, bool)
        for i in range(N):
            for j in (0, 1, 2, 7, 3, 4, 5, 10):
                foot[12 * N + 12 * i + j] = True
        dyn = np.zeros(p, bool); dyn[:12 * N] = True
        d4 = solve_red(r1, r2, r3, r4)
        for step in range(1, 3):
            e = rhs - Kk @ d4
            e1k = np.where(foot, e[:nz], 0.0); e4k = np.where(dyn, e[nz + 2 * m:], 0.0)
            d4 = d4 + solve_red(e1k, e[nz:nz + m], e[nz + m:nz + 2 * m], e4k)
            out[f"kernelform_ref{step}"] = d4[:nz].copy()
        for tag, use_foot, use_dyn in (("e1all", False, True), ("e4all", True, False)):
            d4 = solve_red(r1, r2, r3, r4)
            e = rhs - Kk @ d4
            e1k = np.where(foot, e[:nz], 0.0) if use_foot else e[:nz]
            e4k = np.where(dyn, e[nz + 2 * m:], 0.0) if use_dyn else e[nz + 2 * m:]
            d4 = d4 + solve_red(e1k, e[nz:nz + m], e[nz + m:nz + 2 * m], e4k)
            out[f"kernelform_{tag}"] = d4[:nz].copy()
        # FP64, rows 2-3 only structured (as the kernel would form them): e2 = r2 - (W ds + dz), e3 = r3 - (G dx + ds - delta dz)
        # the same with exact Phi solves
        d4 = solve_red(r1, r2, r3, r4, lambda v: np.linalg.solve(Phi, v))
        for step in range(1, 4):
            e = (rl - Kl @ d4.astype(np.longdouble)).astype(np.float64)
            d4 = d4 + solve_red(e[:nz], e[nz:nz + m], e[nz + m:nz + 2 * m], e[nz + 2 * m:], lambda v: np.linalg.solve(Phi, v))
            out[f"red4x_ref{step}"] = d4[:nz].copy()
        sc = np.abs(xref).max()
        for k, v in out.items():
            res.setdefault((K, k), []).append(np.abs(v - xref).max() / sc)
    print(f"cond Phi (last env) K={K}: {np.linalg.cond(Phi):.1e}  max Lam {Lam.max():.1e}")
for (K, k), v in res.items():
    print(f"K={K:2d} {k:22s} worst {max(v):.1e} median {np.median(v):.1e}")
