"""GPU parity in stress regimes (tests/_stress.py): flight (every contact force pinned to zero by
both-sided rows), one foot in swing for the whole horizon, large tilt, large RL residuals -- the
HIP step against the oracle at K = 10 and 20 on every env, at the SOLVER_CASES tolerance or 4x the
per-env FP64 floor between the two CPU restatements (sparse LDL^T oracle vs dense LU,
tests/golden/make_stress_floor.py), whichever is larger. Every case runs under each solver path:
"auto" (the fused one-launch register kernel: every horizon 2..32), "lds" (former + the LDS-resident
stage-invariant kernel, pdipm_srbd_kernel, at every horizon) and "general" (the CCS-table kernel)."""
import os

import numpy as np
import pytest
import torch

from biped_pympc_amd import solver
from oracle import oracle
from tests._stress import STRESS_CASES, STRESS_K, stress_workload
from tests._util import rel_err_rows
from tests.test_gpu_parity import SOLVER_CASES, U0_TOL

pytestmark = pytest.mark.gpu
FLOOR = os.path.join(os.path.dirname(__file__), "golden", "dense_floor_stress.npz")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device (run them through gpurun)")


@pytest.mark.parametrize("path", ["auto", "lds", "general"])
@pytest.mark.parametrize("name", sorted(STRESS_CASES))
def test_stress_parity(name, path):
    from biped_pympc_amd import _native
    N, wl = stress_workload(name)
    floor = np.load(FLOOR)
    ins = [torch.from_numpy(a).cuda() for a in wl.inputs]
    for K in STRESS_K:
        ref = oracle.mpc_solve(N, K, wl.inputs, y0=1.0)
        with _native.solver_path(path):
            out = [t.cpu().numpy() for t in solver.mpc_solve(ins, N, K, y0=1.0)]
        assert out[1].min() > 0.0 and out[2].min() > 0.0, "iterate left the interior"
        for k, v in enumerate("xszy"):
            assert np.all(np.isfinite(out[k])), (K, v)
            err = rel_err_rows(out[k], ref[k])
            tol = np.maximum(dict(SOLVER_CASES)[K], 4.0 * floor[f"{name}_K{K}_{v}"])
            bad = np.flatnonzero(err > tol)
            assert bad.size == 0, (K, v, err[bad], tol[bad])
        if K == 10:
            u = slice(12 * N, 12 * N + 12)
            assert rel_err_rows(out[0][:, u], ref[0][:, u]).max() <= U0_TOL
