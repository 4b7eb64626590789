"""Per-problem status word (SURVEY.md 5 failure detection; include/srbd_mpc.h SRBD_STATUS_*).

The reference detects nothing per problem (its only guards are the clamps, sparse_pdipm_solver.py
:466-467,501-515), so the word is new API. Its bits 0 (non-finite result) and 1 (step length at its
1e-12 floor in the last iteration) are computed by the oracle with the same definition
(oracle/srbd_oracle.c oracle_pdipm_st) and compared env by env; bit 2 (general fallback) is tested in
tests/test_gpu_parity.py::test_mixed_batch_routes_non_invariant_qps_to_the_general_kernel.
Asking for the word must not change a single bit of the solution.
"""
import numpy as np
import pytest
import torch

from biped_pympc_amd import _native, solver
from biped_pympc_amd.utils.synthetic import make_workload
from oracle import oracle

pytestmark = pytest.mark.gpu

PATHS = ["auto", "lds", "general"]


def _cuda(arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


@pytest.mark.parametrize("N", [1, 5, 10, 20, 32])
@pytest.mark.parametrize("path", PATHS)
def test_status_clean_batch_is_zero_and_changes_nothing(N, path):
    B, K = 48, 10
    wl = make_workload(B, N, seed=300 + N, random_gait=True)
    ins = _cuda(wl.inputs)
    st = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    with _native.solver_path(path):
        bufs_a = solver.MPCSolveBuffers.allocate(N, B)
        bufs_b = solver.MPCSolveBuffers.allocate(N, B)
        a = solver.mpc_solve(ins, N, K, 1.0, buffers=bufs_a)
        b = solver.mpc_solve(ins, N, K, 1.0, buffers=bufs_b, status=st)
    torch.cuda.synchronize()
    for k in range(6):
        assert torch.equal(a[k], b[k]), k
    ref_st = np.zeros(B, np.int32)
    oracle.mpc_solve(N, K, wl.inputs, y0=1.0, status=ref_st)
    assert not ref_st.any()  # bits 0-1 and the oracle's own LDL-failure bit 3 all clear
    assert np.array_equal(st.cpu().numpy(), ref_st)


@pytest.mark.parametrize("N", [1, 10, 20])
@pytest.mark.parametrize("path", PATHS)
def test_status_flags_planted_nan(N, path):
    B, K = 16, 5
    wl = make_workload(B, N, seed=400 + N)
    inputs = [a.copy() for a in wl.inputs]
    inputs[0][3, 2] = np.nan      # x0 of env 3
    inputs[3][7, 12 * N - 1] = np.inf  # x_ref of env 7
    st = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    with _native.solver_path(path):
        solver.mpc_solve(_cuda(inputs), N, K, 1.0, buffers=solver.MPCSolveBuffers.allocate(N, B), status=st)
    torch.cuda.synchronize()
    ref_st = np.zeros(B, np.int32)
    oracle.mpc_solve(N, K, inputs, y0=1.0, status=ref_st)
    got = st.cpu().numpy()
    assert not (np.delete(ref_st, [3, 7]) & oracle.STATUS_LDL_FAIL).any()  # the checker itself did not fail
    assert (ref_st[[3, 7]] & _native.STATUS_NONFINITE).all()
    assert np.array_equal(got & _native.STATUS_NONFINITE, ref_st & _native.STATUS_NONFINITE)
    assert not (np.delete(got, [3, 7])).any()


@pytest.mark.parametrize("N", [5, 10, 20])
@pytest.mark.parametrize("path", PATHS)
def test_status_flags_stalled_warm_start(N, path):
    """A warm start far outside the feasible set with s = z = 1e-8 (all slacks at their clamp):
    the first combined step length sits at its 1e-12 floor (oracle and GPU agree env by env)."""
    B, K = 12, 1
    wl = make_workload(B, N, seed=500 + N)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    rng = np.random.default_rng(N)
    x = rng.normal(size=(B, 24 * N)) * 1e3
    x[B // 2:] = 0.0  # the second half starts cold: no flag
    s = np.full((B, 16 * N), 1e-8)
    z = np.full((B, 16 * N), 1e-8)
    s[B // 2:] = np.maximum(d[B // 2:], 1.0)
    z[B // 2:] = 1.0
    y = np.zeros((B, 14 * N))
    ins = [H, G, A, f, d, b, x, s, z, y]
    ref_st = np.zeros(B, np.int32)
    oracle.pdipm(N, K, ins, status=ref_st)
    st = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    with _native.solver_path(path):
        solver.pdipm(_cuda(ins[:6]), _cuda(ins[6:]), N, K, status=st)
    torch.cuda.synchronize()
    assert not (ref_st & oracle.STATUS_LDL_FAIL).any()  # the checker's factorisation did not fail
    assert (ref_st[:B // 2] == _native.STATUS_STEP_FLOOR).all() and not ref_st[B // 2:].any()
    assert np.array_equal(st.cpu().numpy(), ref_st)


def test_status_from_ccs_entry_and_controller_step():
    """srbd_pdipm_ex's _ccs init (init_mode 2) and srbd_mpc_step_ex report the word too."""
    from biped_pympc_amd.utils.synthetic import make_controller
    N, K, B = 10, 10, 32
    wl = make_workload(B, N, seed=9)
    H, f, A, b, G, d = oracle.qp_former(N, wl.inputs)
    st = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    x0 = torch.zeros((B, 24 * N), dtype=torch.float64, device="cuda")
    solver.pdipm_ccs(_cuda([H, G, A, f, d, b]), x0, N, K, status=st)
    torch.cuda.synchronize()
    assert not st.cpu().numpy().any()
    c = make_controller(B, N, seed=10, device="cuda", n_iter=K)
    c.status = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    wrench, _ = c.run()
    torch.cuda.synchronize()
    assert torch.isfinite(wrench).all()
    assert not c.status.cpu().numpy().any()
