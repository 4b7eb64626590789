"""Torch-facing API over libsrbd_mpc.so (extended C-ABI, caller's current HIP stream).

PyTorch supplies device memory and the stream only; all arithmetic runs in the HIP kernels.
Tensors are batched row-major ``(B, nnz)`` FP64 on the GPU, exactly the CusADi layout
(reference ``biped_pympc/cusadi/src/CusadiFunction.py:71-76``).
"""
from __future__ import annotations


import torch

from biped_pympc_amd import _native
from biped_pympc_amd.layout import Dims


def _stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check_batch(tensors, widths, B: int, what: str):
    for i, (t, w) in enumerate(zip(tensors, widths)):
        if t is None:
            continue
        if not t.is_cuda or t.dtype != torch.float64:
            raise TypeError(f"{what}: input {i} must be a CUDA float64 tensor")
        if t.device.index != torch.cuda.current_device():  # launches go to the current device's stream
            raise ValueError(f"{what}: input {i} is on {t.device}, the current device is "
                             f"cuda:{torch.cuda.current_device()}")
        if t.numel() != B * w:
            raise ValueError(f"{what}: input {i} has {t.numel()} elements, expected {B}x{w}")
        if not t.is_contiguous():
            raise ValueError(f"{what}: input {i} must be contiguous (CusADi row layout)")


def qp_former(inputs: list[torch.Tensor], N: int, outputs: list[torch.Tensor] | None = None):
    """17 former inputs -> [H, f, A, b, G, d] nonzeros (B, nnz) (srbd_constraints.py:20-81)."""
    d = Dims(N)
    B = inputs[0].shape[0]
    _check_batch(inputs, d.former_in_nnz, B, "qp_former")
    if outputs is None:
        outputs = [torch.empty((B, w), dtype=torch.float64, device=inputs[0].device)
                   for w in d.former_out_nnz]
    _check_batch(outputs, d.former_out_nnz, B, "qp_former outputs")
    L = _native.lib()
    rc = L.srbd_qp_former(N, B, _native.ptr_array([t.data_ptr() for t in inputs]),
                          _native.ptr_array([t.data_ptr() for t in outputs]), _stream_ptr())
    _native.check(rc, "srbd_qp_former")
    return outputs


def _check_status(status, B: int, what: str):
    """status: None, or an int32 (B,) CUDA tensor on the current device for the per-problem status
    word (include/srbd_mpc.h SRBD_STATUS_*: 1 non-finite result, 2 step length at its floor in the
    last iteration, 4 general fallback taken)."""
    if status is None:
        return None
    if (not status.is_cuda or status.dtype != torch.int32 or status.numel() != B or not status.is_contiguous()
            or status.device.index != torch.cuda.current_device()):
        raise ValueError(f"{what}: status must be a contiguous int32 CUDA tensor of {B} elements on the current device")
    return status.data_ptr()


def _alloc_solver_outputs(B: int, N: int, device) -> list[torch.Tensor]:
    return [torch.empty((B, w), dtype=torch.float64, device=device) for w in Dims(N).solver_out_nnz]


def pdipm(qp: list[torch.Tensor], iterate: list[torch.Tensor] | None, N: int, n_iter: int,
          y0: float = 1.0, outputs: list[torch.Tensor] | None = None, status: torch.Tensor | None = None):
    """Sparse PDIPM, n_iter Mehrotra iterations (sparse_pdipm_solver.py:357-534).

    qp: [Q_val, G_val, A_val, f, h, b]; iterate: [x, s, z, y] or None for the GPU caller's cold
    start (x=0, s=max(h,1), z=1, y=y0; mpc_controller_cusadi.py:138-141).
    Returns [x, s, z, y, residuals(4), mu(1)]; ``status`` (int32 (B,), optional) receives the
    per-problem status word.
    """
    d = Dims(N)
    B = qp[0].shape[0]
    ins = list(qp) + (list(iterate) if iterate is not None else [None] * 4)
    _check_batch(ins, d.solver_in_nnz, B, "pdipm")
    if outputs is None:
        outputs = _alloc_solver_outputs(B, N, qp[0].device)
    _check_batch(outputs, d.solver_out_nnz, B, "pdipm outputs")
    L = _native.lib()
    ptrs = _native.ptr_array([t.data_ptr() if t is not None else 0 for t in ins])
    outp = _native.ptr_array([t.data_ptr() for t in outputs])
    st = _check_status(status, B, "pdipm")
    if st is not None:
        rc = L.srbd_pdipm_ex(N, n_iter, B, 1 if iterate is None else 0, float(y0), ptrs, outp, st, _stream_ptr())
    elif iterate is None:
        rc = L.srbd_pdipm_cold(N, n_iter, B, float(y0), ptrs, outp, _stream_ptr())
    else:
        rc = L.srbd_pdipm(N, n_iter, B, ptrs, outp, _stream_ptr())
    _native.check(rc, "srbd_pdipm")
    return outputs


def pdipm_ccs(qp: list[torch.Tensor], x_init: torch.Tensor, N: int, n_iter: int,
              outputs: list[torch.Tensor] | None = None, status: torch.Tensor | None = None):
    """The reference's ``_ccs`` solver (sparse_pdipm_solver_ccs, sparse_pdipm_solver.py:4-35): n_iter
    Mehrotra iterations from x = x_init, s = max(h - G x_init, 1), z = 1, y = 0
    (initialize_pdipm_variables, :537-558). qp: [Q_val, G_val, A_val, f, h, b]; x_init (B, 24N).
    Returns [x, s, z, y, residuals(4), mu(1)] (the reference Function returns x)."""
    d = Dims(N)
    B = qp[0].shape[0]
    ins = list(qp) + [x_init, None, None, None]
    _check_batch(ins, d.solver_in_nnz, B, "pdipm_ccs")
    if outputs is None:
        outputs = _alloc_solver_outputs(B, N, qp[0].device)
    _check_batch(outputs, d.solver_out_nnz, B, "pdipm_ccs outputs")
    ptrs = _native.ptr_array([t.data_ptr() if t is not None else 0 for t in ins])
    outp = _native.ptr_array([t.data_ptr() for t in outputs])
    st = _check_status(status, B, "pdipm_ccs")
    if st is not None:
        rc = _native.lib().srbd_pdipm_ex(N, n_iter, B, 2, 0.0, ptrs, outp, st, _stream_ptr())
    else:
        rc = _native.lib().srbd_pdipm_ccs(N, n_iter, B, ptrs, outp, _stream_ptr())
    _native.check(rc, "srbd_pdipm_ccs")
    return outputs


class MPCSolveBuffers:
    """Preallocated device buffers for repeated ``mpc_solve`` calls (no allocation per step).

    ``outputs`` are allocated up front; the QP ``workspace`` (H, f, A, b, G, d: 18 KB per env at
    N = 10) only on first use -- the two-kernel form, ``keep_qp`` or ``qp_views`` -- since the fused
    step never writes it (at 8192 envs it is 148 MB of HBM the default path would hold for nothing)."""

    def __init__(self, N: int, B: int, device, outputs: list, workspace: torch.Tensor | None = None):
        dev = torch.device(device)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.N, self.B, self.device, self.outputs = N, B, dev, outputs
        self._workspace = workspace

    @classmethod
    def allocate(cls, N: int, B: int, device="cuda") -> "MPCSolveBuffers":
        return cls(N, B, device, _alloc_solver_outputs(B, N, device))

    @property
    def workspace_allocated(self) -> bool:
        return self._workspace is not None

    @property
    def workspace(self) -> torch.Tensor:
        if self._workspace is None:
            n = _native.lib().srbd_mpc_workspace_doubles(self.N, self.B)
            self._workspace = torch.empty(max(n, 1), dtype=torch.float64, device=self.device)
        return self._workspace

    def qp_views(self) -> list[torch.Tensor]:
        """[H, f, A, b, G, d] views into the workspace (filled by the former)."""
        d = Dims(self.N)
        out, o = [], 0
        for w in d.former_out_nnz:
            out.append(self.workspace[o:o + self.B * w].view(self.B, w))
            o += self.B * w
        return out


def mpc_solve(former_inputs: list[torch.Tensor], N: int, n_iter: int, y0: float = 1.0,
              buffers: MPCSolveBuffers | None = None, fused: bool = True, keep_qp: bool = False,
              status: torch.Tensor | None = None):
    """qp_former + cold-started PDIPM in one stream with no host synchronisation.

    Equivalent to the GPU caller's step (mpc_controller_cusadi.py:99-169) with the Newton
    iteration count as a runtime argument. Returns [x, s, z, y, residuals, mu].
    ``fused`` (default): one kernel forms the QP in registers / LDS and solves it
    (``srbd_mpc_solve_fused``; the register-resident step kernel at every N in 2..32, the
    LDS-resident step kernel at N = 1): no QP data reaches memory, unless ``keep_qp`` (then f, b, d go to their
    ``buffers.workspace`` slots); ``False`` runs the former and the solver as two kernels with the
    full QP in the workspace. Both give the same bits. ``status`` (int32 (B,), optional) receives
    the per-problem status word.
    """
    d = Dims(N)
    B = former_inputs[0].shape[0]
    _check_batch(former_inputs, d.former_in_nnz, B, "mpc_solve")
    if buffers is None or buffers.B != B or buffers.N != N:
        buffers = MPCSolveBuffers.allocate(N, B, former_inputs[0].device)
    _check_batch(buffers.outputs, d.solver_out_nnz, B, "mpc_solve outputs")
    if buffers.device != former_inputs[0].device:
        raise ValueError(f"mpc_solve: buffers on {buffers.device}, inputs on {former_inputs[0].device}")
    L = _native.lib()
    # the fused kernel runs under the auto solver path (any horizon); otherwise the former writes the
    # whole QP into the workspace for the solver kernel
    one_kernel = fused and _native.current_solver_path() == 0
    args = (N, n_iter, B, float(y0), _native.ptr_array([t.data_ptr() for t in former_inputs]),
            buffers.workspace.data_ptr() if (keep_qp or not one_kernel) else None,
            _native.ptr_array([t.data_ptr() for t in buffers.outputs]))
    st = _check_status(status, B, "mpc_solve")
    if st is not None:  # the two-kernel form runs under srbd_mpc_solve_fused_ex's non-auto branch alike
        if not fused and one_kernel:
            raise ValueError("mpc_solve: status with fused=False needs a non-auto solver path")
        rc = L.srbd_mpc_solve_fused_ex(*args, st, _stream_ptr())
    else:
        rc = (L.srbd_mpc_solve_fused if fused else L.srbd_mpc_solve)(*args, _stream_ptr())
    _native.check(rc, "srbd_mpc_solve")
    return buffers.outputs
