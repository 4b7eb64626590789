"""Shared helpers for the parity tests (compare against the oracle; never used by the product)."""
import numpy as np


def rel_err(a, b) -> float:
    """max |a - b| / max(max |b|, 1e-300) over the whole array (norm-wise relative error)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = max(float(np.abs(b).max()) if b.size else 0.0, 1e-300)
    return float(np.abs(a - b).max()) / scale if b.size else 0.0


def rel_err_rows(a, b) -> np.ndarray:
    """Per-env norm-wise relative error (rows of a batched (B, n) array)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    scale = np.maximum(np.abs(b).max(axis=1), 1e-300)
    return np.abs(a - b).max(axis=1) / scale


def dense_floor_env(N: int, K: int, ins, e: int):
    """FP64 floor of one env's solve: per-output (x, s, z, y) relative distance between the two CPU
    restatements of the solver -- the C oracle (sparse LDL^T) and oracle/pdipm_dense.py (dense LU) --
    on the solver inputs `ins` (10 batched arrays) of env e. A GPU result within a few times this is at
    the precision the problem admits (used where a fixed tolerance meets an ill-conditioned env)."""
    from oracle import oracle
    from oracle.pdipm_dense import pdipm_dense
    one = [np.asarray(a)[e:e + 1] for a in ins]
    ref = oracle.pdipm(N, K, one)
    den = pdipm_dense(N, K, *[a[0] for a in one])
    return [float(rel_err_rows(np.asarray(den[k])[None], ref[k]).max()) for k in range(4)]
