"""GPU parity: HIP kernels (through the C-ABI) vs the CPU oracle on identical seeded inputs.

Mirrors the reference's only parity harness, ``biped_pympc/cusadi/run_cusadi_function_test.py``
(batched device evaluation vs per-env CPU evaluation, error per output), with the oracle in place
of CasADi (absent here; see oracle/srbd_oracle.c). Tolerances are norm-wise relative errors
(max |gpu - oracle| / max |oracle| per output); the bar from BASELINE.json is 1e-4 on the QP
solution, the former is checked at 1e-12.
"""
import numpy as np
import pytest
import torch

from biped_pympc_amd import layout, solver
from biped_pympc_amd.utils.synthetic import make_workload, solver_init
from oracle import oracle
from tests._util import rel_err, rel_err_rows

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a ROCm device (run them through gpurun)")


def _cuda(arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


@pytest.mark.parametrize("N,random_gait", [(10, False), (10, True), (20, False), (1, False), (32, True)])
def test_former_matches_oracle(N, random_gait):
    wl = make_workload(256, N, seed=11 + N, random_gait=random_gait, residuals=random_gait)
    ref = oracle.qp_former(N, wl.inputs)
    out = solver.qp_former(_cuda(wl.inputs), N)
    torch.cuda.synchronize()
    for k, (o, r) in enumerate(zip(out, ref)):
        err = rel_err(o.cpu().numpy(), r)
        assert err <= 1e-12, f"output {k} rel err {err:.3e}"


# (K, tolerance on x/s/z/y): two FP64 factorisation orders of the same KKT drift apart as the
# barrier closes (oracle-vs-dense-numpy noise floor, tests/test_oracle.py); u0 keeps <= 1e-6.
SOLVER_CASES = [(1, 1e-9), (5, 1e-7), (10, 1e-6), (20, 1e-4)]


@pytest.mark.parametrize("N", [10, 20])
@pytest.mark.parametrize("K,tol", SOLVER_CASES)
def test_solver_matches_oracle(N, K, tol):
    B = 64
    wl = make_workload(B, N, seed=100 + K, random_gait=(K % 2 == 0))
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    x, s, z, y = solver_init(d, N)
    ins = [H, G, A, f, d, b, x, s, z, y]
    ref = oracle.pdipm(N, K, ins)
    out = solver.pdipm(_cuda(ins[:6]), _cuda(ins[6:]), N, K)
    torch.cuda.synchronize()
    out = [o.cpu().numpy() for o in out]
    names = ["x", "s", "z", "y", "residuals", "mu"]
    for k in range(4):
        errs = rel_err_rows(out[k], ref[k])
        assert np.all(np.isfinite(out[k])), names[k]
        assert errs.max() <= tol, f"{names[k]}: worst env rel err {errs.max():.3e} (median {np.median(errs):.1e})"
    u0_err = rel_err_rows(out[0][:, 12 * N:12 * N + 12], ref[0][:, 12 * N:12 * N + 12])
    assert u0_err.max() <= max(tol, 1e-6)


def test_cold_start_matches_explicit_init():
    N, B, K = 10, 128, 10
    wl = make_workload(B, N, seed=7)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    x, s, z, y = solver_init(d, N, y0=1.0)
    qp = _cuda([H, G, A, f, d, b])
    warm = solver.pdipm(qp, _cuda([x, s, z, y]), N, K)
    cold = solver.pdipm(qp, None, N, K, y0=1.0)
    torch.cuda.synchronize()
    for a, c in zip(warm, cold):
        assert torch.equal(a, c)


def test_mpc_solve_end_to_end():
    """Fused stream (former -> cold PDIPM, K = 10) vs the oracle's full GPU-caller step."""
    N, B, K = 10, 256, 10
    wl = make_workload(B, N, seed=3)
    ref = oracle.mpc_solve(N, K, wl.inputs, y0=1.0)
    out = solver.mpc_solve(_cuda(wl.inputs), N, K, y0=1.0)
    torch.cuda.synchronize()
    x = out[0].cpu().numpy()
    u_gpu, u_ref = x[:, 12 * N:12 * N + 12], ref[0][:, 12 * N:12 * N + 12]
    assert rel_err_rows(u_gpu, u_ref).max() <= 1e-6
    assert rel_err_rows(x, ref[0]).max() <= 1e-6


def test_iteration_schedule_composes():
    """4 calls x 5 iterations (the reference GPU schedule, mpc_controller_cusadi.py:144-169) equal
    one call x 20 iterations: the solver keeps no hidden state."""
    N, B = 10, 64
    wl = make_workload(B, N, seed=5)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    qp = _cuda([H, G, A, f, d, b])
    it = _cuda(list(solver_init(d, N)))
    one = solver.pdipm(qp, it, N, 20)
    cur = it
    for _ in range(4):
        o = solver.pdipm(qp, cur, N, 5)
        cur = [t.clone() for t in o[:4]]
    torch.cuda.synchronize()
    for a, c in zip(one[:4], cur):
        assert torch.equal(a, c)
