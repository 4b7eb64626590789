"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the
product package ``biped_pympc_amd`` never does. See ``srbd_oracle.c`` for what it restates
(reference ``srbd_constraints.py:20-227``, ``srbd_centroidal_model.py:101-166``,
``sparse_pdipm_solver.py:357-534``) and why parity against CasADi itself is unpinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from biped_pympc_amd import layout

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libsrbd_oracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


_registered: set[int] = set()
_I32P = ctypes.POINTER(ctypes.c_int)


def _iptr(a: np.ndarray):
    return a.ctypes.data_as(_I32P)


def register(N: int) -> None:
    if N in _registered:
        return
    Hp, Hi = layout.ccs_H(N)
    Ap, Ai = layout.ccs_A(N)
    Gp, Gi = layout.ccs_G(N)
    arrs = [np.ascontiguousarray(a, np.int32) for a in (Hp, Hi, Ap, Ai, Gp, Gi)]
    rc = lib().oracle_set_pattern(ctypes.c_int(N), *[_iptr(a) for a in arrs])
    if rc != 0:
        raise RuntimeError(f"oracle_set_pattern failed for N={N}")
    _registered.add(N)


def _ptr_array(arrays):
    arr_t = ctypes.c_void_p * len(arrays)
    return arr_t(*[a.ctypes.data for a in arrays])


def _as_batch(a, width: int, B: int) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(a, np.float64).reshape(B, width))
    return a


def qp_former(N: int, inputs, B: int | None = None, nthreads: int = 0):
    """inputs: 17 arrays shaped (B, nnz_in[i]) (or 1-D for a single env). Returns 6 (B, nnz) arrays."""
    register(N)
    d = layout.Dims(N)
    single = np.asarray(inputs[0]).ndim == 1
    if B is None:
        B = 1 if single else np.asarray(inputs[0]).shape[0]
    ins = [_as_batch(a, w, B) for a, w in zip(inputs, d.former_in_nnz)]
    outs = [np.zeros((B, w)) for w in d.former_out_nnz]
    rc = lib().oracle_qp_former_batch(ctypes.c_int(N), ctypes.c_int(B), _ptr_array(ins),
                                      _ptr_array(outs), ctypes.c_int(nthreads))
    if rc < 0:
        raise RuntimeError("oracle_qp_former_batch failed")
    if rc > 0:
        raise AssertionError("qp_former Jacobian has nonzeros outside the registered CCS pattern")
    return [o[0] for o in outs] if single else outs


# status bit the oracle alone sets: its sparse LDL^T met a zero pivot (srbd_oracle.c ORACLE_STATUS_LDL_FAIL)
STATUS_LDL_FAIL = 8


def _status_arg(status):
    return None if status is None else status.ctypes.data_as(_I32P)


ORDERS = {"md": 0, "amd": 1}  # the KKT elimination order: exact minimum degree (the checker), CasADi's AMD


def pdipm(N: int, n_iter: int, inputs, B: int | None = None, nthreads: int = 0, status: np.ndarray | None = None,
          order: str = "md"):
    """inputs: Q_val, G_val, A_val, f, h, b, x, s, z, y as (B, nnz). Returns x, s, z, y, res(4), mu(1).
    status: an int32 (B,) array receiving the per-problem status word (srbd_oracle.c); with it a
    failed factorisation is reported there (STATUS_LDL_FAIL) instead of raising. order: "md" (exact
    minimum degree, the checker) or "amd" (approximate minimum degree, the order of CasADi's ldl)."""
    register(N)
    d = layout.Dims(N)
    single = np.asarray(inputs[0]).ndim == 1
    if B is None:
        B = 1 if single else np.asarray(inputs[0]).shape[0]
    ins = [_as_batch(a, w, B) for a, w in zip(inputs, d.solver_in_nnz)]
    outs = [np.zeros((B, w)) for w in d.solver_out_nnz]
    rc = lib().oracle_pdipm_batch_ord(ctypes.c_int(N), ctypes.c_int(n_iter), ctypes.c_int(B), _ptr_array(ins),
                                      _ptr_array(outs), ctypes.c_int(nthreads), _status_arg(status),
                                      ctypes.c_int(ORDERS[order]))
    if rc < 0:
        raise RuntimeError("oracle_pdipm_batch failed")
    if rc > 0:
        raise FloatingPointError("oracle LDL hit a zero pivot")
    return [o[0] for o in outs] if single else outs


def mpc_solve(N: int, n_iter: int, former_inputs, y0: float = 1.0, B: int | None = None,
              nthreads: int = 0, status: np.ndarray | None = None):
    """Former + GPU-caller init (x=0, s=max(d,1), z=1, y=y0) + n_iter iterations (status: as pdipm)."""
    register(N)
    d = layout.Dims(N)
    if B is None:
        B = np.asarray(former_inputs[0]).reshape(-1, 12).shape[0]
    ins = [_as_batch(a, w, B) for a, w in zip(former_inputs, d.former_in_nnz)]
    outs = [np.zeros((B, w)) for w in d.solver_out_nnz]
    rc = lib().oracle_mpc_solve_batch(ctypes.c_int(N), ctypes.c_int(n_iter), ctypes.c_double(y0),
                                      ctypes.c_int(B), _ptr_array(ins), _ptr_array(outs),
                                      ctypes.c_int(nthreads), _status_arg(status))
    if rc < 0:
        raise RuntimeError("oracle_mpc_solve_batch failed")
    if rc > 0:
        raise FloatingPointError("oracle former/LDL failure")
    return outs


def kkt_stats(N: int, order: str = "md") -> dict:
    register(N)
    n, nk, nl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    if lib().oracle_kkt_stats_ord(ctypes.c_int(N), ctypes.c_int(ORDERS[order]), ctypes.byref(n), ctypes.byref(nk),
                                  ctypes.byref(nl)):
        raise RuntimeError("oracle_kkt_stats failed")
    return {"n": n.value, "nnz_kkt": nk.value, "nnz_L": nl.value}


def kkt_order(N: int, order: str = "md") -> np.ndarray:
    """The KKT elimination order (perm[k] = the row eliminated k-th) under `order`."""
    register(N)
    n = kkt_stats(N, order)["n"]
    perm = np.zeros(n, np.int32)
    if lib().oracle_kkt_order(ctypes.c_int(N), ctypes.c_int(ORDERS[order]), _iptr(perm)) != n:
        raise RuntimeError("oracle_kkt_order failed")
    return perm


def amd_order(n: int, Kp, Ki) -> np.ndarray:
    """srbd_oracle.c amd_order (CasADi's ldl ordering, restated) of a symmetric CSC pattern."""
    Kp = np.ascontiguousarray(Kp, np.int32)
    Ki = np.ascontiguousarray(Ki, np.int32)
    perm = np.zeros(n, np.int32)
    if lib().oracle_amd_order(ctypes.c_int(n), _iptr(Kp), _iptr(Ki), _iptr(perm)):
        raise RuntimeError("oracle_amd_order failed")
    return perm
