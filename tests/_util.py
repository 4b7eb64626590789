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
