"""The CCS contract between qp_former and the solver (no GPU needed).

The reference never writes the sparsity down: it is whatever CasADi's structural jacobian of the
RK4 model yields (srbd_constraints.py:83-227) and get_ccs() hands to the solver
(generate_solver_function.py:69-76). Here it is derived three independent ways and all must agree:
  1. closed-form rules (biped_pympc_amd/layout.py),
  2. structural dependency propagation through the literal RK4 of forward_dynamics (below),
  3. the offset maps the HIP kernels use (srbd_pattern_ccs in libsrbd_mpc.so),
and the oracle's numerical AD Jacobian must have no nonzero outside it.
"""
import ctypes
import os

import numpy as np
import pytest

from biped_pympc_amd import layout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dyn_dependency():
    """Boolean dependency of forward_dynamics outputs on [x(12); u(12)]
    (srbd_centroidal_model.py:150-166): R, I^-1 full symbolic 3x3, skew has a zero diagonal."""
    D = np.zeros((12, 24), bool)
    D[0:3, 6:9] = True  # euler_dot = R @ omega
    for r in range(3):
        D[3 + r, 9 + r] = True  # p_dot = v
    tq = np.zeros((3, 24), bool)  # torque = skew(rL) fL + skew(rR) fR + mL + mR
    for k in range(3):
        for j in range(3):
            if j != k:
                tq[k, 12 + j] = True
                tq[k, 15 + j] = True
        tq[k, 18 + k] = True
        tq[k, 21 + k] = True
    D[6:9] = tq.any(axis=0)  # I^-1 @ torque (full)
    for r in range(3):
        D[9 + r, 12 + r] = True
        D[9 + r, 15 + r] = True
    return D


def _rk4_dependency():
    D = _dyn_dependency()
    ident = np.zeros((12, 24), bool)
    ident[np.arange(12), np.arange(12)] = True

    def f(dep_state):  # dependency of f(state, u) given the state's dependency sets
        out = np.zeros((12, 24), bool)
        for r in range(12):
            for c in np.nonzero(D[r])[0]:
                out[r] |= dep_state[c] if c < 12 else (np.arange(24) == c)
        return out

    k1 = f(ident)
    k2 = f(ident | k1)
    k3 = f(ident | k2)
    k4 = f(ident | k3)
    return ident | k1 | k2 | k3 | k4


def _structural_ccs_A(N):
    dep = _rk4_dependency()
    nz, p = 24 * N, 14 * N
    M = np.zeros((p, nz), bool)
    for i in range(N):
        for r in range(12):
            M[12 * i + r, 12 * i + r] = True  # x_{i+1} - ...
            for c in np.nonzero(dep[r])[0]:
                if c < 12:
                    if i >= 1:
                        M[12 * i + r, 12 * (i - 1) + c] = True
                else:
                    M[12 * i + r, 12 * N + 12 * i + (c - 12)] = True
        M[12 * N + 2 * i, 12 * N + 12 * i + 6] = True
        M[12 * N + 2 * i + 1, 12 * N + 12 * i + 9] = True
    colptr = np.concatenate([[0], np.cumsum(M.sum(axis=0))]).astype(np.int32)
    rows = np.concatenate([np.nonzero(M[:, c])[0] for c in range(nz)]).astype(np.int32)
    return colptr, rows


@pytest.mark.parametrize("N", [1, 2, 10, 20, 32])
def test_nnz_counts(N):
    d = layout.Dims(N)
    assert layout.ccs_A(N)[0][-1] == d.nnz_A == 122 * N - 24
    assert layout.ccs_G(N)[0][-1] == d.nnz_G == 28 * N
    assert layout.ccs_H(N)[0][-1] == d.nnz_H == 24 * N
    if N == 10:  # the reference's artefact name: mpc_..._240v_140eq_160ineq (mpc_controller_cusadi.py:28)
        assert (d.nz, d.n_eq, d.n_ineq) == (240, 140, 160)
        assert (d.nnz_A, d.nnz_G) == (1196, 280)


@pytest.mark.parametrize("N", [1, 3, 10, 20])
def test_rows_ascending_within_columns(N):
    for cp, ri in (layout.ccs_A(N), layout.ccs_G(N), layout.ccs_H(N)):
        for c in range(len(cp) - 1):
            col = ri[cp[c]:cp[c + 1]]
            assert np.all(np.diff(col) > 0)


@pytest.mark.parametrize("N", [1, 2, 10, 20])
def test_structural_dependency_matches_closed_form(N):
    cp, ri = _structural_ccs_A(N)
    cpl, ril = layout.ccs_A(N)
    assert np.array_equal(cp, cpl)
    assert np.array_equal(ri, ril)


def test_G_pattern_matches_constraint_list():
    # srbd_constraints.py:193-222: per foot 8 rows over (fx, fy, fz, my)
    N = 2
    G = np.zeros((16 * N, 24 * N), bool)
    cp, ri = layout.ccs_G(N)
    for c in range(24 * N):
        G[ri[cp[c]:cp[c + 1]], c] = True
    for i in range(N):
        for f in range(2):
            cols = [12 * N + 12 * i + 3 * f + k for k in range(3)] + [12 * N + 12 * i + 7 + 3 * f]
            expect = {0: [cols[0], cols[2]], 1: [cols[0], cols[2]], 2: [cols[1], cols[2]],
                      3: [cols[1], cols[2]], 4: [cols[2], cols[3]], 5: [cols[2], cols[3]],
                      6: [cols[2]], 7: [cols[2]]}
            for k, cs in expect.items():
                assert sorted(np.nonzero(G[16 * i + 8 * f + k])[0].tolist()) == sorted(cs)


@pytest.mark.parametrize("N", [1, 2, 10, 20, 32])
def test_kernel_offset_maps_match_layout(N):
    from biped_pympc_amd import _native
    L = _native.lib()
    P = ctypes.POINTER(ctypes.c_int)
    for which, (cp_ref, ri_ref) in enumerate((layout.ccs_H(N), layout.ccs_A(N), layout.ccs_G(N))):
        cp = np.zeros(24 * N + 1, np.int32)
        ri = np.zeros(len(ri_ref), np.int32)
        nnz = L.srbd_pattern_ccs(N, which, cp.ctypes.data_as(P), ri.ctypes.data_as(P))
        assert nnz == len(ri_ref)
        assert np.array_equal(cp, cp_ref) and np.array_equal(ri, ri_ref)


@pytest.mark.parametrize("N", [2, 10])
def test_stage_tables_address_the_right_entries(N):
    t = layout.stage_tables(N)
    cp, ri = layout.ccs_A(N)
    cols = np.repeat(np.arange(24 * N), np.diff(cp))
    for i in range(N):
        for r in range(12):
            off = 36 * i + t["P"][r] if i < N - 1 else 36 * (N - 1) + r
            assert (ri[off], cols[off]) == (12 * i + r, 12 * i + r)
        ub = int(t["ubase"]) + 86 * i
        for j in range(12):
            for q, row in enumerate(layout.S_U[j]):
                off = ub + t["NU"][j][q]
                assert (ri[off], cols[off]) == (12 * i + row, 12 * N + 12 * i + j)
        assert (ri[ub + t["E6"]], cols[ub + t["E6"]]) == (12 * N + 2 * i, 12 * N + 12 * i + 6)
        assert (ri[ub + t["E9"]], cols[ub + t["E9"]]) == (12 * N + 2 * i + 1, 12 * N + 12 * i + 9)


def test_dense_roundtrip():
    rng = np.random.default_rng(0)
    N = 3
    cp, ri = layout.ccs_A(N)
    v = rng.normal(size=(5, len(ri)))
    dense = layout.to_dense(v, cp, ri, (14 * N, 24 * N))
    assert np.array_equal(layout.from_dense(dense, cp, ri), v)
    assert np.count_nonzero(dense[0]) == len(ri)


def test_sii_entry_order_covers_each_class_once():
    """The S_ii build's lane -> entry table (csrc/srbd_common.hpp kSiiOrder): the 21 dense x dense
    entries first, then the 57 with a sparse index, each packed-lower entry exactly once, and the
    LDS store conflicts it was chosen for (scripts/sii_order.py)."""
    import re
    import sys
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from sii_order import dense_cost, sparse_cost
    src = open(os.path.join(ROOT, "biped_pympc_amd", "csrc", "srbd_common.hpp")).read()
    body = re.search(r"kSiiOrder\[78\] = \{([^}]*)\}", src).group(1)
    order = [(int(v) & 15, int(v) >> 4) for v in body.split(",")]
    assert len(order) == 78 and len(set(order)) == 78 and all(r >= c for r, c in order)
    sparse = lambda e: (e[0] % 6 >= 3) + (e[1] % 6 >= 3)
    assert all(sparse(e) == 0 for e in order[:21]) and all(sparse(e) > 0 for e in order[21:])
    assert dense_cost(order[:21]) <= 5 and sparse_cost(order[21:]) <= 1

