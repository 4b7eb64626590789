"""The refinement step's two ways of updating dz, ds, emulated on the CPU against the long-double answer
(CPU host; diagnostics for DESIGN.md 3.3).

    python scripts/refine_form_emu.py

The GPU kernels eliminate the KKT of sparse_pdipm_solver.py:412-439 as ds, dz -> dx (Phi) -> dy (Schur
complement of the dynamics rows), then refine once against all four rows. This emulates that elimination
densely in FP64 (numpy), with one refinement step in two forms:
  "re-formed": dz = VV' + Lambda G dx, ds = -r_s' - G dx + delta dz from the WHOLE refined dx (rounds 1-6);
  "additive":  dz += q + Lambda G c_x, ds += e3 + delta q + (delta Lambda - 1) G c_x from the correction.
and runs the PDIPM iterations of the failing envs of round 6's campaigns with each, against
scripts/extended_precision_check.py's long-double restatement. Lambda = W / (1 + delta W) multiplies the
rounding of G dx (eps |G| |dx|) in the re-formed dz: at z / s = 6e5 that is the 1e-9 the GPU showed.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
LD = np.longdouble
DELTA = 1e-8

# (seed, env, _ccs sequence): failing envs of the round-6 campaigns (general, LDS-resident, register paths)
ENVS = [(53625, 76, True), (53795, 12, True), (52137, 238, False), (54145, 162, False), (55300, 116, False)]


def kkt(N, ins):
    from biped_pympc_amd import layout
    Hv, Gv, Av, f, h, b, x, s, z, y = (np.asarray(v, np.float64) for v in ins)
    nz, m, p = 24 * N, 16 * N, 14 * N
    H = layout.to_dense(Hv, *layout.ccs_H(N), (nz, nz))
    G = layout.to_dense(Gv, *layout.ccs_G(N), (m, nz))
    A = layout.to_dense(Av, *layout.ccs_A(N), (p, nz))
    rx, re, rs = H @ x + f + G.T @ z + A.T @ y, A @ x - b, G @ x + s - h
    W = (1.0 / s) * z + DELTA
    n = nz + 2 * m + p
    K = np.zeros((n, n))
    K[:nz, :nz] = H + DELTA * np.eye(nz)
    K[:nz, nz + m:nz + 2 * m] = G.T
    K[:nz, nz + 2 * m:] = A.T
    K[nz:nz + m, nz:nz + m] = np.diag(W)
    K[nz:nz + m, nz + m:nz + 2 * m] = np.eye(m)
    K[nz + m:nz + 2 * m, :nz] = G
    K[nz + m:nz + 2 * m, nz:nz + m] = np.eye(m)
    K[nz + m:nz + 2 * m, nz + m:nz + 2 * m] = -DELTA * np.eye(m)
    K[nz + 2 * m:, :nz] = A
    K[nz + 2 * m:, nz + 2 * m:] = -DELTA * np.eye(p)
    return K, (H, G, A, W, nz, m, p), rx, re, rs


def eliminate(parts, r):
    """ds, dz -> dx -> dy elimination of K d = r (the GPU's order; dense inverses)."""
    H, G, A, W, nz, m, p = parts
    r1, r2, r3, r4 = r[:nz], r[nz:nz + m], r[nz + m:nz + 2 * m], r[nz + 2 * m:]
    D = 1 + DELTA * W
    VV, Lam = (r2 - W * r3) / D, W / D
    Phi_inv = np.linalg.inv(H + DELTA * np.eye(nz) + G.T @ (Lam[:, None] * G))
    t = Phi_inv @ (r1 - G.T @ VV)
    dy = np.linalg.inv(A @ Phi_inv @ A.T + DELTA * np.eye(p)) @ (A @ t - r4)
    dx = t - Phi_inv @ (A.T @ dy)
    dz = VV + Lam * (G @ dx)
    return np.concatenate([dx, r3 - G @ dx + DELTA * dz, dz, dy]), VV, Lam


def refined(K, parts, r, form):
    H, G, A, W, nz, m, p = parts
    d, VV, Lam = eliminate(parts, r)
    e = r - K @ d
    c, _, _ = eliminate(parts, e)
    if form == "additive":
        return d + c
    e2, e3 = e[nz:nz + m], e[nz + m:nz + 2 * m]
    q = (e2 - W * e3) / (1 + DELTA * W)
    dx = d[:nz] + c[:nz]
    gd = G @ dx
    dz = (VV + q) + Lam * gd
    ds = (r[nz + m:nz + 2 * m] + e3) - gd + DELTA * dz
    return np.concatenate([dx, ds, dz, d[nz + 2 * m:] + c[nz + 2 * m:]])


def step(v, dv):
    c = dv < 0
    a = -v / np.where(c, dv, -1.0)
    return max(min(1.0, 0.99 * np.fmin.reduce(np.where(c, a, 0.0) + np.where(c, 0.0, 1.0))), 1e-12)


def pdipm(N, K_it, ins, form):
    Hv, Gv, Av, f, h, b, x, s, z, y = (np.asarray(v, np.float64) for v in ins)
    nz, m = 24 * N, 16 * N
    for _ in range(K_it):
        K, parts, rx, re, rs = kkt(N, [Hv, Gv, Av, f, h, b, x, s, z, y])
        si = 1.0 / s
        r = np.concatenate([-rx, -(si * (s * z)), -rs, -re])
        a = refined(K, parts, r, form)
        dsa, dza = a[nz:nz + m], a[nz + m:nz + 2 * m]
        ap, ad = step(s, dsa), step(z, dza)
        mu = s @ z / m
        sigma = ((s + ap * dsa) @ (z + ad * dza) / m / mu) ** 3
        r[nz:nz + m] = -(si * (s * z)) + -(si * (s * z + dsa * dza - sigma * mu))
        d = refined(K, parts, r, form)
        dx, ds, dz, dy = d[:nz], d[nz:nz + m], d[nz + m:nz + 2 * m], d[nz + 2 * m:]
        apc, adc = step(s, ds), step(z, dz)
        x, s = x + apc * dx, np.fmax(s + apc * ds, 1e-8)
        z, y = np.fmax(z + adc * dz, 1e-8), y + adc * dy
    return x, s, z, y


def main():
    import importlib
    import extended_precision_check as epc
    for seed, env, ccs in ENVS:
        os.environ["FUZZ_CCS"] = "1" if ccs else "0"
        import parity_fuzz
        pf = importlib.reload(parity_fuzz)
        N, K, B, entry, path, kw, y0, extra = pf.replay_all(seed)[seed]
        _, ins = pf.case_inputs(seed, N, K, B, entry, kw, y0, extra)
        one = [np.asarray(a)[env] for a in ins]
        _, ex = epc.pdipm_ld(N, K, *one)
        for form in ("re-formed", "additive"):
            out = pdipm(N, K, one, form)
            e = [float(np.abs(o.astype(LD) - x_[0]).max() / np.abs(x_[0]).max()) for o, x_ in zip(out, ex)]
            print(f"seed {seed} env {env:3d} N{N} K{K:2d} {entry:5s} {path:7s} {form:9s}: "
                  + " ".join(f"{n} {v:.1e}" for n, v in zip("xszy", e)), flush=True)


if __name__ == "__main__":
    main()
