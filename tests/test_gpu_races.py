"""Race detection for the device code (the reference has none; a sanitizer build of the
device code is not available on this pool -- GPU AddressSanitizer and XNACK runs are refused).

The kernels synchronise through LDS barriers (multi-wave QPs), wavefront-scope fences in place of
`s_waitcnt` drains (one-wave QPs), DPP wait states (audited statically by test_isa_hazards.py), and in
the in-launch general fallback through lock words on a scratch pool in HBM shared by every workgroup.
A missing wait or fence changes results only under some wave interleavings, so every kernel family is
launched repeatedly under different timing -- alone, beside a concurrent FP64 GEMM on another stream
(which takes CUs and shifts wave placement), with a different batch layout around the same QPs, and in
a child process with every launch serialised (AMD_SERIALIZE_KERNEL=3) -- and each launch must
reproduce the first bit for bit. Batches of 2048 + 300 QPs leave the second wave of workgroups partial,
so co-residency differs between the two rounds of a launch.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from biped_pympc_amd import _native, solver
from biped_pympc_amd.utils.synthetic import make_workload
from tests.test_gpu_parity import _cuda, _mixed_inputs

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = 2348
REPS = 6


def _noise():
    """A concurrent FP64 GEMM on its own stream (bounded values: fixed operands, out= buffer)."""
    st = torch.cuda.Stream()
    a = torch.randn(3072, 3072, dtype=torch.float64, device="cuda") / 64
    c = torch.empty_like(a)

    def run():
        with torch.cuda.stream(st):
            for _ in range(3):
                torch.mm(a, a, out=c)
    return run


def _repeat_identical(fn):
    """fn() -> list of output tensors; REPS launches alone and REPS beside the noise GEMM, all equal
    to the first launch's bits."""
    first = [t.clone() for t in fn()]
    noise = _noise()
    for r in range(2 * REPS):
        if r % 2:
            noise()
        out = fn()
        torch.cuda.synchronize()
        for k, (a, b) in enumerate(zip(first, out)):
            assert torch.equal(a, b), f"launch {r} (noise={bool(r % 2)}): output {k} differs"
    return first


@pytest.mark.parametrize("N", [1, 10, 20, 23, 28])
def test_fused_step_is_deterministic_under_contention(N):
    """One-wave (N = 10), two-wave (20), three-wave (23), four-wave (28) register QPs and the
    LDS-resident step kernel (N = 1)."""
    K = 10
    wl = make_workload(B, N, seed=9300 + N, random_gait=True, residuals=True)
    ins = _cuda(wl.inputs)
    first = _repeat_identical(lambda: solver.mpc_solve(ins, N, K, y0=1.0))
    # the same QPs at other batch positions, next to other QPs: the rows are the same bits
    perm = torch.randperm(B, generator=torch.Generator().manual_seed(N)).cuda()
    other = solver.mpc_solve([t[perm].contiguous() for t in ins], N, K, y0=1.0)
    torch.cuda.synchronize()
    for a, b in zip(first, other):
        assert torch.equal(a[perm], b)


@pytest.mark.parametrize("N,path", [(10, "auto"), (20, "auto"), (10, "lds"), (20, "lds"), (10, "general")])
def test_ccs_solver_is_deterministic_under_contention(N, path):
    """The CCS solver kernels (register, LDS-resident, general) on a stage-invariant batch."""
    K = 5
    wl = make_workload(B, N, seed=9400 + N, random_gait=True)
    qp = solver.qp_former(_cuda(wl.inputs), N)
    sol_qp = [qp[0], qp[4], qp[2], qp[1], qp[5], qp[3]]
    with _native.solver_path(path):
        _repeat_identical(lambda: solver.pdipm(sol_qp, None, N, K, 1.0))


def test_fallback_pool_is_deterministic_under_contention():
    """Mixed batch (two thirds not stage-invariant) on a 3-slot pool: the fallback QPs queue on the
    lock words and hand slots over between workgroups; the noise GEMM changes who waits for whom."""
    _native.set_scratch_slots(3)
    try:
        ins, _ = _mixed_inputs(10, 600, seed=95)
        qp, it = _cuda(ins[:6]), _cuda(ins[6:])
        _repeat_identical(lambda: solver.pdipm(qp, it, 10, 5))
    finally:
        _native.set_scratch_slots(0)
    _native.prepare_device()  # the default pool again, before any capture test


_SERIAL_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from biped_pympc_amd import solver
from biped_pympc_amd.utils.synthetic import make_workload
out = {}
for N in (10, 20):
    wl = make_workload(int(sys.argv[3]), N, seed=9300 + N, random_gait=True, residuals=True)
    x = solver.mpc_solve([torch.from_numpy(a).cuda() for a in wl.inputs], N, 10, 1.0)
    torch.cuda.synchronize()
    for k, t in enumerate(x):
        out[f"N{N}_{k}"] = t.cpu().numpy()
np.savez(sys.argv[2], **out)
print("serial ok")
"""


def test_serialized_launches_give_the_same_bits(tmp_path):
    """AMD_SERIALIZE_KERNEL=3 (every launch waits for the previous one, before and after) in a child
    process vs this process's own launches: the same bits at N = 10 and N = 20."""
    path = tmp_path / "serial.npz"
    env = dict(os.environ, AMD_SERIALIZE_KERNEL="3", AMD_SERIALIZE_COPY="3")
    r = subprocess.run([sys.executable, "-c", _SERIAL_CHILD, ROOT, str(path), str(B)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    got = np.load(path)
    for N in (10, 20):
        wl = make_workload(B, N, seed=9300 + N, random_gait=True, residuals=True)
        x = solver.mpc_solve(_cuda(wl.inputs), N, 10, 1.0)
        torch.cuda.synchronize()
        for k, t in enumerate(x):
            assert np.array_equal(t.cpu().numpy(), got[f"N{N}_{k}"]), (N, k)
