"""The reference GPU caller's QP schedule, issued through the drop-in ``CusadiFunction``.

``MPCControllerCusadi.run`` (reference ``biped_pympc/convex_mpc/mpc_controller_cusadi.py:99-172``)
does not call one fused solve: it calls the ``qp_former`` library once, rebuilds the six dense
outputs, initialises the iterate with a dense ``(B,16N,24N) @ (B,24N,1)`` product, then calls the
5-iteration ``sparse_pdipm_multiple_iterations`` library four times, each call followed by four
``getDenseOutput`` rebuilds and ``clone()`` of the iterate. Every ``evaluate`` is blocking
(``generateCUDACode.py:176-182``). A user who keeps that controller and only swaps the libraries
(INTEGRATION.md option A) runs exactly this; ``ReferenceQPSchedule`` issues it against our
libraries so the bench can time it (``dropin_step``) beside the one-launch fused step.

``lean=True`` is the same call sequence with the reference's host-side glue trimmed to what the
solver needs: the sparse outputs feed the next call directly (no dense rebuilds, no bmm: the
cold-start s = max(d, 1) is what ``G @ 0`` gives), so it measures the libraries, not torch glue.
"""
from __future__ import annotations

import torch

from biped_pympc_amd.cusadi.CusadiFunction import CusadiFunction
from biped_pympc_amd.cusadi.function import pdipm_function, qp_former_function


class ReferenceQPSchedule:
    def __init__(self, N: int, num_envs: int, n_calls: int = 4, iters_per_call: int = 5, lean: bool = False):
        self.N, self.num_envs, self.n_calls, self.lean = N, int(num_envs), n_calls, lean
        self.qp_former = CusadiFunction(qp_former_function(N), self.num_envs)
        self.qp_solver = CusadiFunction(pdipm_function(N, iters_per_call), self.num_envs)

    def run(self, former_inputs: list[torch.Tensor]) -> torch.Tensor:
        """17 former inputs (B, nnz_in) FP64 -> the solution x (B, 24N) after n_calls solver calls."""
        B = self.num_envs
        self.qp_former.evaluate(former_inputs)  # mpc_controller_cusadi.py:99
        out = self.qp_former.outputs_sparse
        H_col, G_col, A_col = (t.double().contiguous() for t in (out[0], out[4], out[2]))  # :119-121
        f_col = out[1].reshape(B, -1, 1).double().contiguous()  # :122-124
        d_col = out[5].reshape(B, -1, 1).double().contiguous()
        b_col = out[3].reshape(B, -1, 1).double().contiguous()
        if self.lean:
            x = torch.zeros(B, 24 * self.N, device=H_col.device, dtype=torch.float64)
            s = torch.clamp(d_col.reshape(B, -1), min=1.0)  # max(d - G 0, 1)
            z = torch.ones_like(s)
            y = torch.ones(B, 14 * self.N, device=H_col.device, dtype=torch.float64)
        else:
            for k in range(6):  # :103-108, dense H, f, A, b, G, d
                dense = self.qp_former.getDenseOutput(k)
                if k == 4:
                    G = dense
                elif k == 5:
                    d = dense.squeeze(-1)
            x = torch.zeros(B, 24 * self.N, device=H_col.device, dtype=torch.float64)  # :138-141
            s = torch.maximum(d - (G @ x.unsqueeze(2)).squeeze(2), torch.ones_like(d))
            z = torch.ones(B, 16 * self.N, device=H_col.device, dtype=torch.float64)
            y = torch.ones(B, 14 * self.N, device=H_col.device, dtype=torch.float64)
        for _ in range(self.n_calls):  # :144-169
            ins = [H_col, G_col, A_col, f_col, d_col, b_col] + [
                t.double().reshape(B, -1, 1).contiguous() for t in (x, s, z, y)]
            self.qp_solver.evaluate(ins)
            if self.lean:  # the next evaluate zeroes the outputs it reads from: own copies
                x, s, z, y = (self.qp_solver.outputs_sparse[k].clone() for k in range(4))
            else:
                x, s, z, y = (self.qp_solver.getDenseOutput(k).reshape(B, -1).clone().detach() for k in range(4))
        return x.clone().detach()  # :172
