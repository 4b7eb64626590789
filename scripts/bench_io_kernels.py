"""Time the caller-side kernels of the MPC step against the HBM roof (GPU box):
srbd_prepare_inputs, the standalone qp_former, srbd_u0_wrench and srbd_dense_scatter (H, A, G).

python scripts/bench_io_kernels.py [B]   -> one line per kernel: ms, algorithmic bytes, GB/s
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from biped_pympc_amd import _native, layout, solver  # noqa: E402
from biped_pympc_amd.controller import (DesiredStateData, MPCConf, MPCControllerHIP,  # noqa: E402
                                        StateEStimatorData, dense_scatter, inverse_index)
from biped_pympc_amd.utils.synthetic import make_workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = 10
REPS = 20
d = layout.Dims(N)


def timed(fn):
    s = torch.cuda.current_stream()
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(REPS):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / REPS


def report(name, ms, nbytes):
    print(f"{name:28s} {ms * 1e3:9.2f} us   {nbytes / 1e6:8.2f} MB   {nbytes / (ms * 1e-3) / 1e9:8.1f} GB/s "
          f"({100 * nbytes / (ms * 1e-3) / 8e12:.1f} % of 8 TB/s)")


c = MPCControllerHIP(B, "cuda", 2, MPCConf())
se, ds = StateEStimatorData(2, B, "cuda"), DesiredStateData(B, "cuda")
se.foot_position[:, 0, 1], se.foot_position[:, 1, 1] = 0.1, -0.1
c.set_state_estimate_data(se)
c.set_desired_state_data(ds)
keep = []
p = c._prep_struct(keep)
L = _native.lib()
outs = _native.ptr_array([t.data_ptr() for t in c.former_inputs])
ms = timed(lambda: L.srbd_prepare_inputs(N, B, ctypes.byref(p), outs, solver._stream_ptr()))
report("prepare_inputs", ms, B * (4 * (3 * 4 + 9 + 6 + 3 + 3 + 1 + 1 + 3 + 3 + 4 + 1 + 2 + 2) + 8 * sum(d.former_in_nnz)))

wl = make_workload(B, N, seed=1)
ins = [torch.from_numpy(a).cuda() for a in wl.inputs]
qp = solver.qp_former(ins, N)
ms = timed(lambda: solver.qp_former(ins, N, outputs=qp))
report("qp_former", ms, B * 8 * (sum(d.former_in_nnz) + sum(d.former_out_nnz)))

x = torch.randn(B, d.nz, dtype=torch.float64, device="cuda")
rot = se.rotation_body.contiguous()
w = torch.empty(B, 2, 6, device="cuda")
ms = timed(lambda: L.srbd_u0_wrench(N, B, x.data_ptr(), rot.data_ptr(), w.data_ptr(), solver._stream_ptr()))
report("u0_wrench", ms, B * (12 * 8 + 9 * 4 + 12 * 4))

for name, (cp, ri), shape, vals in (("H", layout.ccs_H(N), (d.nz, d.nz), qp[0]),
                                    ("A", layout.ccs_A(N), (d.n_eq, d.nz), qp[2]),
                                    ("G", layout.ccs_G(N), (d.n_ineq, d.nz), qp[4])):
    rows, cols = layout.triplet(cp, ri)
    inv = inverse_index(rows, cols, shape, "cuda")
    out = torch.empty(B, *shape, dtype=torch.float64, device="cuda")
    ms = timed(lambda: dense_scatter(vals, inv, shape, out))
    report(f"dense_scatter {name} {shape[0]}x{shape[1]}", ms, B * 8 * (shape[0] * shape[1] + len(rows)))
