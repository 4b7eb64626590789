"""Synthetic batched SRBD-MPC workloads, numpy FP64, seeded.

The inputs are laid out exactly as the reference GPU caller hands them to ``qp_former``
(``biped_pympc/convex_mpc/mpc_controller_cusadi.py:54-95``): one ``(B, nnz_in[i])`` row-major
array per input. Two caller quirks are reproduced on purpose:
  * ``R_body`` is flattened row-major by the caller (``:58``) and decoded column-major by CasADi,
    so the former effectively sees R^T;
  * ``contact_table`` (B, N, 2) is flattened row-major (``:65``) and decoded as a column-major N x 2.
Pass ``contact_layout="casadi"`` to lay the contact table out the way CasADi indexes it instead.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from biped_pympc_amd.layout import Dims

HECTOR_MASS = 13.856  # core/robot/hector.py:34
HECTOR_MU = 1.0  # core/robot/hector.py:38
HECTOR_I_BODY = np.diag([0.5413, 0.5200, 0.0691])  # core/robot/hector.py:35-37
Q_DEFAULT = np.array([150, 150, 250, 100, 100, 250, 1, 1, 5, 10, 10, 1], np.float64)  # configuration.py:45
R_DEFAULT = np.array([1e-5] * 6 + [1e-4] * 6, np.float64)  # configuration.py:50
DT_MPC = 0.025  # configuration.py:38


def rot_zyx(roll, pitch, yaw) -> np.ndarray:
    """R = Rz(yaw) Ry(pitch) Rx(roll), batched (B, 3, 3)."""
    cr, sr = np.cos(roll), np.sin(roll)
    cp, sp = np.cos(pitch), np.sin(pitch)
    cy, sy = np.cos(yaw), np.sin(yaw)
    R = np.empty(np.shape(roll) + (3, 3))
    R[..., 0, 0] = cy * cp
    R[..., 0, 1] = cy * sp * sr - sy * cr
    R[..., 0, 2] = cy * sp * cr + sy * sr
    R[..., 1, 0] = sy * cp
    R[..., 1, 1] = sy * sp * sr + cy * cr
    R[..., 1, 2] = sy * sp * cr - cy * sr
    R[..., 2, 0] = -sp
    R[..., 2, 1] = cp * sr
    R[..., 2, 2] = cp * cr
    return R


def mpc_gait_table(phase: np.ndarray, ssp: np.ndarray, dsp: np.ndarray, horizon: int) -> np.ndarray:
    """Contact table (B, horizon, 2) int32, restating ``GaitGenerator.mpc_gait``
    (``biped_pympc/core/gait/gait_generator.py:216-252``; durations per env as (B, 2) ints)."""
    ssp = np.asarray(ssp, np.int64)
    dsp = np.asarray(dsp, np.int64)
    cycle = (ssp + dsp).sum(axis=1)  # :50
    # (gait_phase * gait_cycle_length).int(): float32 product truncated toward zero
    t0 = (np.asarray(phase, np.float32) * cycle.astype(np.float32)).astype(np.int64)
    steps = (t0[:, None] + np.arange(horizon)[None, :]) % cycle[:, None]
    s1, d0, s0 = ssp[:, 1:2], dsp[:, 0:1], ssp[:, 0:1]
    ph1 = steps < s1
    ph2 = (steps >= s1) & (steps < s1 + d0)
    ph3 = (steps >= s1 + d0) & (steps < s1 + d0 + s0)
    tab = np.zeros(steps.shape + (2,), np.int32)
    tab[..., 0][ph1] = 1
    tab[..., 0][ph2] = 1
    tab[..., 1][ph2] = 1
    tab[..., 1][ph3] = 1
    rest = ~(ph1 | ph2 | ph3)
    tab[..., 0][rest] = 1
    tab[..., 1][rest] = 1
    return tab


@dataclass
class Workload:
    N: int
    B: int
    inputs: list  # 17 arrays (B, nnz_in[i]) float64, qp_former input order
    R_body: np.ndarray  # (B, 3, 3) true body rotation
    contact: np.ndarray  # (B, N, 2) int32 (before flattening)
    meta: dict


def make_workload(B: int, N: int = 10, seed: int = 0, random_gait: bool = False,
                  residuals: bool = False, contact_layout: str = "reference",
                  dt: float = DT_MPC, tilt: float = 0.15, residual_scale: float = 0.5,
                  contact_override: np.ndarray | None = None) -> Workload:
    """SURVEY 8d synthetic robots. Stress knobs (defaults = the SURVEY distributions): ``tilt`` bounds
    roll and pitch, ``residual_scale`` is the std of the RL residual accelerations (with
    ``residuals``), ``contact_override`` (B, N, 2) replaces the contact schedule (e.g. flight)."""
    rng = np.random.default_rng(seed)
    d = Dims(N)
    roll = rng.uniform(-tilt, tilt, B)
    pitch = rng.uniform(-tilt, tilt, B)
    yaw = rng.uniform(-math.pi, math.pi, B)
    R = rot_zyx(roll, pitch, yaw)
    Iw = R @ HECTOR_I_BODY[None] @ np.swapaxes(R, 1, 2)
    body = np.stack([rng.uniform(-1, 1, B), rng.uniform(-1, 1, B),
                     0.55 + rng.uniform(-0.03, 0.03, B)], axis=1)
    off_l = np.stack([rng.uniform(-0.05, 0.05, B), np.full(B, 0.10), np.full(B, -0.55)], axis=1)
    off_r = np.stack([rng.uniform(-0.05, 0.05, B), np.full(B, -0.10), np.full(B, -0.55)], axis=1)
    foot_l = body + np.einsum("bij,bj->bi", R, off_l)
    foot_r = body + np.einsum("bij,bj->bi", R, off_r)
    omega = rng.normal(0.0, 0.2, (B, 3))
    vel = rng.normal(0.0, 0.3, (B, 3))
    x0 = np.concatenate([np.stack([roll, pitch, yaw], 1), body, omega, vel], axis=1)
    # reference trajectory, base_controller.py:213-257 (non-stationary branch)
    vb = np.stack([rng.uniform(-1, 1, B), rng.uniform(-1, 1, B), np.zeros(B)], axis=1)
    wz = rng.uniform(-1, 1, B)
    vw = np.einsum("bij,bj->bi", R, vb)
    tb = dt * np.arange(N)[None, :]
    xref = np.zeros((B, N, 12))
    xref[:, :, 2] = yaw[:, None] + wz[:, None] * tb
    xref[:, :, 3] = body[:, 0:1] + vw[:, 0:1] * tb
    xref[:, :, 4] = body[:, 1:2] + vw[:, 1:2] * tb
    xref[:, :, 5] = 0.55
    xref[:, :, 8] = wz[:, None]
    xref[:, :, 9] = vw[:, 0:1]
    xref[:, :, 10] = vw[:, 1:2]
    if random_gait:
        ssp = rng.integers(3, 7, (B, 2))
        dsp = rng.integers(0, 3, (B, 2))
        phase = rng.uniform(0.0, 1.0, B).astype(np.float32)
        contact = mpc_gait_table(phase, ssp, dsp, N)
    else:
        contact = np.ones((B, N, 2), np.int32)
        ssp = dsp = phase = None
    if contact_override is not None:
        contact = np.asarray(contact_override, np.int32).reshape(B, N, 2)
    if contact_layout == "reference":
        ct_flat = contact.reshape(B, 2 * N).astype(np.float64)  # row-major, as the caller does
    elif contact_layout == "casadi":
        ct_flat = np.swapaxes(contact, 1, 2).reshape(B, 2 * N).astype(np.float64)
    else:
        raise ValueError(contact_layout)
    a_lin = rng.normal(0.0, residual_scale, (B, 3)) if residuals else np.zeros((B, 3))
    a_ang = rng.normal(0.0, residual_scale, (B, 3)) if residuals else np.zeros((B, 3))
    inputs = [
        x0,
        np.ones((B, 12 * N)),
        np.ones((B, 12 * N)),
        xref.reshape(B, 12 * N),
        np.full((B, 1), dt),
        np.full((B, 1), HECTOR_MASS),
        np.full((B, 1), HECTOR_MU),
        R.reshape(B, 9),  # row-major flatten (mpc_controller_cusadi.py:58)
        Iw.reshape(B, 9),
        body,
        foot_l,
        foot_r,
        ct_flat,
        np.tile(Q_DEFAULT, (B, 1)),
        np.tile(R_DEFAULT, (B, 1)),
        a_lin,
        a_ang,
    ]
    inputs = [np.ascontiguousarray(a, np.float64) for a in inputs]
    for a, w in zip(inputs, d.former_in_nnz):
        assert a.shape == (B, w), (a.shape, w)
    meta = {"seed": seed, "random_gait": random_gait, "residuals": residuals,
            "contact_layout": contact_layout, "R_body_flatten": "row-major (caller quirk)",
            "dt": dt}
    return Workload(N=N, B=B, inputs=inputs, R_body=R, contact=contact, meta=meta)


def solver_init(d_vec: np.ndarray, N: int, y0: float = 1.0):
    """GPU-caller iterate init (mpc_controller_cusadi.py:138-141): x=0, s=max(d,1), z=1, y=y0."""
    B = d_vec.shape[0]
    dims = Dims(N)
    x = np.zeros((B, dims.nz))
    s = np.maximum(d_vec, 1.0)
    z = np.ones((B, dims.n_ineq))
    y = np.full((B, dims.n_eq), y0)
    return x, s, z, y


def make_controller(B: int, N: int = 10, seed: int = 0, device="cuda", n_iter: int = 10):
    """An MPCControllerHIP over B synthetic robots (float32 state estimate / command / gait as the
    reference data classes hold them, SURVEY 8d distributions, device-side gait schedule): the
    controller-step workload of bench.py."""
    import torch

    from biped_pympc_amd.controller import DesiredStateData, MPCConf, MPCControllerHIP, StateEStimatorData
    rng = np.random.default_rng(seed)
    eul = np.stack([rng.uniform(-0.15, 0.15, B), rng.uniform(-0.15, 0.15, B), rng.uniform(-math.pi, math.pi, B)], 1)
    R = rot_zyx(eul[:, 0], eul[:, 1], eul[:, 2])
    pos = np.stack([rng.uniform(-1, 1, B), rng.uniform(-1, 1, B), 0.55 + rng.uniform(-0.03, 0.03, B)], 1)
    feet = np.stack([pos + np.einsum("bij,j->bi", R, [0.0, 0.10, -0.55]),
                     pos + np.einsum("bij,j->bi", R, [0.0, -0.10, -0.55])], 1)
    f32 = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(device)  # noqa: E731
    c = MPCControllerHIP(B, device, 2, MPCConf(horizon_length=N, pdipm_iterations=n_iter))
    se = StateEStimatorData(2, B, device)
    se.root_euler, se.root_position, se.rotation_body, se.foot_position = f32(eul), f32(pos), f32(R), f32(feet)
    se.root_angular_velocity_w = f32(rng.normal(0, 0.2, (B, 3)))
    se.root_velocity_w = f32(rng.normal(0, 0.3, (B, 3)))
    ds = DesiredStateData(B, device)
    ds.desired_velocity_b = f32(np.stack([rng.uniform(-1, 1, B), rng.uniform(-1, 1, B), np.zeros(B)], 1))
    ds.desired_angular_velocity_b = f32(np.stack([np.zeros(B), np.zeros(B), rng.uniform(-1, 1, B)], 1))
    ds.desired_height = f32(0.55 + rng.uniform(-0.02, 0.02, B))
    c.set_state_estimate_data(se)
    c.set_desired_state_data(ds)
    c.set_gait(torch.from_numpy(rng.uniform(0, 1, B).astype(np.float32)),
               torch.from_numpy(rng.integers(3, 7, (B, 2))), torch.from_numpy(rng.integers(0, 3, (B, 2))))
    return c
