"""Diagnostic (GPU box): per-env relative wrench error of the HIP MPC solve vs the oracle at several
iteration counts, on the batch of tests/test_controller.py::test_controller_step_matches_oracle_pipeline.
Shows the truncated-IPM path sensitivity of a few near-degenerate envs (large mid-path differences
that vanish once converged). SRBD_LIB selects another build of libsrbd_mpc.so to compare.

python scripts/diag_path_sensitivity.py
"""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from tests.test_controller import random_robot, _controller
from oracle import mpc_io, oracle
N, B = 10, 128
st, cmd, ctrl, params, gait_args, table = random_robot(B, 21, N, gait=True)
ins, _ = mpc_io.prepare_inputs(N, st, cmd, ctrl, params, gait=gait_args)
from biped_pympc_amd import solver
dins = [torch.from_numpy(a).cuda() for a in ins]
for K in (10, 15, 20, 30):
    xg = solver.mpc_solve(dins, N, K, 1.0)[0].cpu().numpy()
    xo = oracle.mpc_solve(N, K, ins, y0=1.0)[0]
    wg = mpc_io.u0_wrench(N, xg, st["rotation_body"]); wo = mpc_io.u0_wrench(N, xo, st["rotation_body"])
    err = np.abs(wg - wo).max(axis=(1, 2)) / np.maximum(np.abs(wo).max(axis=(1, 2)), 1.0)
    dx = np.abs(xg - xo).max(axis=1) / np.maximum(np.abs(xo).max(axis=1), 1.0)
    o = np.argsort(-err)[:4]
    print(f"K={K}: wrench err top {[(int(i), float(err[i])) for i in o]}  median {np.median(err):.2e}  x-rel top {float(dx.max()):.2e} env {int(dx.argmax())}")
