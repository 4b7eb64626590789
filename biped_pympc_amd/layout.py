"""SRBD-MPC QP layout: dimensions and the CCS sparsity contract between qp_former and the solver.

The reference fixes these patterns implicitly: ``qp_former`` is a CasADi SX Function whose outputs
carry the *structural* sparsity of ``casadi.hessian`` / ``casadi.jacobian``
(reference ``biped_pympc/casadi/srbd_constraints.py:20-81,83-142,144-227``), and
``generate_solver_function.py:61-76,107-114`` hands ``H/A/G.sparsity().get_ccs()`` to
``sparse_pdipm_multiple_iterations`` (``sparse_pdipm_solver.py:357-383``), which rebuilds the
matrices with ``sx_from_ccs`` (``:571-591``). CasADi is absent here, so the pattern is restated in
closed form and cross-checked in ``tests/`` against a structural
dependency analysis of the literal RK4 model (``oracle/``) and against dense reconstruction.

Conventions (CasADi CCS, ``sparse_pdipm_solver.py:561-591``): values are column-major, row indices
ascending inside each column.

Decision vector ``z = [x_1 .. x_N, u_0 .. u_{N-1}]`` (``srbd_constraints.py:22-26,102-105``):
  * state  x_k (k = 1..N), component j  ->  12*(k-1) + j
  * input  u_i (i = 0..N-1), component j ->  12*N + 12*i + j
Equality rows: dynamics of stage i -> 12*i + r (r = 0..11); x-moment rows -> 12*N + 2*i + {0,1}.
Inequality rows: stage i, foot f (0 = left, 1 = right), constraint k -> 16*i + 8*f + k.
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache

import numpy as np

NX = 12
NU = 12
F_MAX = 500.0  # srbd_constraints.py:31
LT = 0.07  # srbd_constraints.py:161
LH = 0.04  # srbd_constraints.py:162
BETA = 1e-8  # generate_solver_function.py:112
DELTA = 1e-8  # sparse_pdipm_solver.py:416

# Per-column row sets of one stage.
# S_x(j): rows of stage k's dynamics block touched by x_k[j] through -A_d.
S_X = tuple(
    (j,) if j <= 5 else ((0, 1, 2, j) if j <= 8 else (j - 6, j)) for j in range(12)
)
# S_u(j): rows of stage i's dynamics block touched by u_i[j] through -B_d.
S_U = tuple(
    (0, 1, 2, 3 + j, 6, 7, 8, 9 + j)
    if j <= 2
    else ((0, 1, 2, j, 6, 7, 8, 6 + j) if j <= 5 else (0, 1, 2, 6, 7, 8))
    for j in range(12)
)
# G per-stage column patterns: u column j -> rows (stage-local, 0..15).
# srbd_constraints.py:193-222: per foot f (offset 8f, force cols 3f..3f+2, m_y col 7+3f):
#   k0 -fx - mu fz, k1 fx - mu fz, k2 -fy - mu fz, k3 fy - mu fz,
#   k4 -lt fz - my, k5 -lh fz + my, k6 -fz, k7 fz - Fmax*contact
G_COLS = {
    0: (0, 1), 1: (2, 3), 2: (0, 1, 2, 3, 4, 5, 6, 7), 7: (4, 5),
    3: (8, 9), 4: (10, 11), 5: (8, 9, 10, 11, 12, 13, 14, 15), 10: (12, 13),
}


@dataclass(frozen=True)
class Dims:
    N: int

    @property
    def nz(self) -> int:  # decision variables
        return 24 * self.N

    @property
    def n_eq(self) -> int:
        return 14 * self.N

    @property
    def n_ineq(self) -> int:
        return 16 * self.N

    @property
    def n_kkt(self) -> int:
        return 70 * self.N

    @property
    def nnz_H(self) -> int:
        return 24 * self.N

    @property
    def nnz_A(self) -> int:
        return 122 * self.N - 24

    @property
    def nnz_G(self) -> int:
        return 28 * self.N

    # qp_former I/O (srbd_constraints.py:77 input order; outputs [H, f, A, b, G, d])
    @property
    def former_in_nnz(self) -> tuple[int, ...]:
        N = self.N
        return (12, 12 * N, 12 * N, 12 * N, 1, 1, 1, 9, 9, 3, 3, 3, 2 * N, 12, 12, 3, 3)

    @property
    def former_out_nnz(self) -> tuple[int, ...]:
        return (self.nnz_H, self.nz, self.nnz_A, self.n_eq, self.nnz_G, self.n_ineq)

    # solver I/O (sparse_pdipm_solver.py:533 input order; outputs x, s, z, y, residuals, mu)
    @property
    def solver_in_nnz(self) -> tuple[int, ...]:
        return (self.nnz_H, self.nnz_G, self.nnz_A, self.nz, self.n_ineq, self.n_eq,
                self.nz, self.n_ineq, self.n_ineq, self.n_eq)

    @property
    def solver_out_nnz(self) -> tuple[int, ...]:
        return (self.nz, self.n_ineq, self.n_ineq, self.n_eq, 4, 1)


FORMER_IN_NAMES = ("x0", "x", "u", "x_ref", "dt", "m", "mu", "R_body", "I_world_inv", "body_pos",
                   "left_foot_pos", "right_foot_pos", "contact_table", "Q", "R",
                   "residual_lin_accel", "residual_ang_accel")
FORMER_OUT_NAMES = ("o0", "o1", "o2", "o3", "o4", "o5")  # CasADi auto-names: H, f, A, b, G, d
SOLVER_IN_NAMES = ("Q_val", "G_val", "A_val", "f", "h", "b", "x", "s", "z", "y")
SOLVER_OUT_NAMES = ("o0", "o1", "o2", "o3", "o4", "o5")


def x_index(N: int, k: int, j: int) -> int:
    """Column of x_k[j], k = 1..N."""
    return 12 * (k - 1) + j


def u_index(N: int, i: int, j: int) -> int:
    """Column of u_i[j], i = 0..N-1."""
    return 12 * N + 12 * i + j


@lru_cache(maxsize=None)
def ccs_A(N: int) -> tuple[np.ndarray, np.ndarray]:
    """(colptr, rowind) of A (14N x 24N)."""
    colptr = [0]
    rows: list[int] = []
    for k in range(1, N + 1):
        for j in range(12):
            col = [12 * (k - 1) + j]
            if k < N:
                col += [12 * k + r for r in S_X[j]]
            rows += col
            colptr.append(len(rows))
    for i in range(N):
        for j in range(12):
            col = [12 * i + r for r in S_U[j]]
            if j == 6:
                col.append(12 * N + 2 * i)
            if j == 9:
                col.append(12 * N + 2 * i + 1)
            rows += col
            colptr.append(len(rows))
    return np.asarray(colptr, np.int32), np.asarray(rows, np.int32)


@lru_cache(maxsize=None)
def ccs_G(N: int) -> tuple[np.ndarray, np.ndarray]:
    """(colptr, rowind) of G (16N x 24N); x columns are empty."""
    colptr = [0] * (12 * N + 1)
    rows: list[int] = []
    for i in range(N):
        for j in range(12):
            rows += [16 * i + r for r in G_COLS.get(j, ())]
            colptr.append(len(rows))
    return np.asarray(colptr, np.int32), np.asarray(rows, np.int32)


@lru_cache(maxsize=None)
def ccs_H(N: int) -> tuple[np.ndarray, np.ndarray]:
    n = 24 * N
    return np.arange(n + 1, dtype=np.int32), np.arange(n, dtype=np.int32)


def ccs_dense_col(n: int) -> tuple[np.ndarray, np.ndarray]:
    """A structurally dense n x 1 column (f, b, d and every vector input)."""
    return np.asarray([0, n], np.int32), np.arange(n, dtype=np.int32)


def triplet(colptr: np.ndarray, rowind: np.ndarray) -> tuple[list[int], list[int]]:
    """CasADi ``Sparsity.get_triplet()``: (rows, cols) in nonzero order."""
    cols = np.repeat(np.arange(len(colptr) - 1), np.diff(colptr))
    return rowind.tolist(), cols.tolist()


def to_dense(values: np.ndarray, colptr: np.ndarray, rowind: np.ndarray, shape) -> np.ndarray:
    """``sx_from_ccs`` (sparse_pdipm_solver.py:571-591) on numbers; batched over leading dims."""
    values = np.asarray(values)
    out = np.zeros(values.shape[:-1] + tuple(shape), values.dtype)
    cols = np.repeat(np.arange(len(colptr) - 1), np.diff(colptr))
    out[..., rowind, cols] = values
    return out


def from_dense(mat: np.ndarray, colptr: np.ndarray, rowind: np.ndarray) -> np.ndarray:
    cols = np.repeat(np.arange(len(colptr) - 1), np.diff(colptr))
    return np.asarray(mat)[..., rowind, cols]


@lru_cache(maxsize=None)
def stage_tables(N: int) -> dict[str, np.ndarray]:
    """Per-stage gather offsets into A_val/G_val used by the HIP solver.

    Every stage's slice of A is addressed as ``base + offset`` with stage-independent offsets
    (the pattern is periodic in the stage index), so the kernel needs only these small tables:
      * ``P[r]``     : +I entry of x_{i+1}[r] in stage-i rows   -> A_val[36*i + P[r]]  (i < N-1)
                       last stage (x_N columns hold only that entry) -> A_val[36*(N-1) + r]
      * ``M[j][t]``  : x_i[j] entries (rows S_X[j][t])          -> A_val[36*(i-1) + M[j][t]]
      * ``NU[j][t]`` : u_i[j] entries (rows S_U[j][t])          -> A_val[36N-24 + 86*i + NU[j][t]]
      * ``E6, E9``   : x-moment rows' entries on u_i[6], u_i[9] -> A_val[36N-24 + 86*i + E]
    (these tables are checked against ``ccs_A`` in tests)."""
    colptr, _ = ccs_A(N)
    P = np.array([colptr[j] for j in range(12)], np.int32)  # stage 0 base
    M = -np.ones((12, 4), np.int32)
    for j in range(12):
        for t in range(len(S_X[j])):
            M[j, t] = colptr[j] + 1 + t  # x_1 column j of stage 1 block, relative to 36*(1-1)
    ubase = int(colptr[12 * N])
    NUt = -np.ones((12, 8), np.int32)
    for j in range(12):
        for t in range(len(S_U[j])):
            NUt[j, t] = int(colptr[12 * N + j]) + t - ubase
    E6 = int(colptr[12 * N + 6]) + len(S_U[6]) - ubase
    E9 = int(colptr[12 * N + 9]) + len(S_U[9]) - ubase
    return {"P": P, "M": M, "NU": NUt, "E6": np.int32(E6), "E9": np.int32(E9),
            "ubase": np.int32(ubase)}
