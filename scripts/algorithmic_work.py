"""Structural (algorithm-independent) work per SRBD QP solve, frozen into bench.py.

Convention: the reference's own algorithm -- a sparse LDL^T of its 70N x 70N KKT
per Newton iteration (sparse_pdipm_solver.py:412-452) under a fill-reducing ordering -- counted
from the symbolic factorisation of the committed CCS pattern:
  F_iter = sum_j (c_j^2 + c_j)              factorisation (c_j = off-diagonal nnz of column j of L)
         + 2 (4 nnz_L + n)                  two solves (affine + corrector)
         + 2 (nz + 2 nnz_G + 2 nnz_A)       residual mat-vecs
         + 6 n + 8 m + 8 n                  rhs / step-length / update vector work
Bytes are the algorithmic HBM traffic of each kernel boundary (FP64, 8 B), inputs read once.
Test tooling: imports the oracle for the symbolic factorisation only.
"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from biped_pympc_amd.layout import Dims  # noqa: E402
from oracle import oracle  # noqa: E402


def work(N: int) -> dict:
    d = Dims(N)
    oracle.register(N)
    st = oracle.kkt_stats(N)
    n = st["n"]
    Lp = np.zeros(n + 1, np.int32)
    oracle.lib().oracle_kkt_lp(ctypes.c_int(N), Lp.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    c = np.diff(Lp).astype(np.int64)
    f_factor = int((c * c + c).sum())
    f_solve = 2 * (4 * st["nnz_L"] + n)
    f_resid = 2 * (d.nz + 2 * d.nnz_G + 2 * d.nnz_A)
    f_vec = 6 * n + 8 * d.n_ineq + 8 * n
    f_iter = f_factor + f_solve + f_resid + f_vec
    former_in = sum(d.former_in_nnz) * 8
    qp = sum(d.former_out_nnz) * 8
    sol_out = sum(d.solver_out_nnz) * 8
    warm = (d.nz + 2 * d.n_ineq + d.n_eq) * 8
    return {
        "N": N, "n_kkt": n, "nnz_kkt": st["nnz_kkt"], "nnz_L": st["nnz_L"],
        "flops_factor": f_factor, "flops_per_iter": f_iter,
        "bytes_former_read": former_in, "bytes_former_write": qp,
        "bytes_pdipm_cold": qp + sol_out,          # reads the QP once, writes x,s,z,y,res,mu
        "bytes_pdipm_warm": qp + warm + sol_out,   # + warm-start iterate (drop-in solver call)
        "bytes_step": former_in + qp + qp + sol_out,  # former -> workspace -> cold PDIPM
        "bytes_fused_min": former_in + sol_out,    # a fully fused kernel's floor
    }


if __name__ == "__main__":
    print(json.dumps({N: work(N) for N in (10, 20)}, indent=1))
