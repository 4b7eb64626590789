"""CPU restatement of the MPC step's caller-side glue (TEST INFRASTRUCTURE ONLY).

Only tests/ import this. It restates, in numpy FP32 with one rounding per torch op (numpy float32
elementwise ops round each operation, as torch's unfused elementwise kernels do):
  * BaseMPCController.compute_knot_points / set_initial_state / compute_reference_trajectory
    (reference biped_pympc/convex_mpc/base_controller.py:166-257);
  * GaitGenerator.mpc_gait (biped_pympc/core/gait/gait_generator.py:216-252) -- pinned against
    tables produced by the reference module itself (tests/golden/gait_reference.npz);
  * the input assembly and the u0 -> foot-wrench tail of MPCControllerCusadi.run
    (biped_pympc/convex_mpc/mpc_controller_cusadi.py:54-95, 186-203).
The 3x3 FP32 products (R v, R I Rᵀ, Rᵀ f) are written as ((a0 b0 + a1 b1) + a2 b2): the reference
runs them as torch bmm, whose reduction order is implementation-defined (results within 1 ulp), so
the kernel and this restatement fix the same order. Parity for these rows is therefore pinned by
the gait fixtures for the contact schedule and unpinned (restatement only) for the FP32 glue.
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def _dot3(m0, m1, m2, v0, v1, v2):
    return (m0 * v0 + m1 * v1) + m2 * v2


def mpc_gait(phase, ssp, dsp, N):
    """gait_generator.py:216-252 for per-env (B,) phase and (B,2) SSP/DSP durations."""
    ssp = np.asarray(ssp, np.int64)
    dsp = np.asarray(dsp, np.int64)
    cyc = (ssp + dsp).sum(axis=1)
    g = (np.asarray(phase, f32) * cyc.astype(f32)).astype(np.int64)  # :223, float32 product, trunc
    st = (g[:, None] + np.arange(N)[None, :]) % cyc[:, None]  # :226-228
    s1, d0, s0 = ssp[:, 1:2], dsp[:, 0:1], ssp[:, 0:1]
    p1 = st < s1
    p2 = (st >= s1) & (st < s1 + d0)
    p3 = (st >= s1 + d0) & (st < s1 + d0 + s0)
    fin = ~(p1 | p2 | p3)
    tab = np.zeros(st.shape + (2,), np.int32)
    tab[..., 0] = (p1 | p2 | fin)
    tab[..., 1] = (p2 | p3 | fin)
    return tab


def prepare_inputs(N, st, cmd, ctrl, params, gait=None, contact_table=None, literal=True):
    """Returns (17 former inputs as float64 arrays, updated controller state dict).

    st: root_euler, root_position, root_angular_velocity_w, root_velocity_w (B,3),
        rotation_body (B,3,3), foot_position (B,2,3); cmd: desired_velocity_b (B,3),
        desired_angular_velocity_b (B,3), desired_height (B); ctrl: world_position_desired (B,3),
        yaw_desired (B), first_run (B) bool; params: dt_mpc (B), residual_lin_accel (B,3),
        residual_ang_accel (B,3), I_body (3,3), mass, mu, Q (12|13), R (12), step_dt (float32);
    gait: (phase (B,), ssp (B,2), dsp (B,2)) or contact_table (B,N,2).
    """
    B = st["root_position"].shape[0]
    rp = st["root_position"].astype(f32)
    eu = st["root_euler"].astype(f32)
    Rm = st["rotation_body"].astype(f32)
    wpd = ctrl["world_position_desired"].astype(f32).copy()
    yaw = ctrl["yaw_desired"].astype(f32).copy()
    fr = ctrl["first_run"].astype(bool).copy()
    # compute_knot_points (:166-176)
    wpd[fr] = rp[fr]
    yaw[fr] = eu[fr, 2]
    fr[:] = False
    # set_initial_state (:201-211)
    x0 = np.concatenate([eu, rp, st["root_angular_velocity_w"].astype(f32),
                         st["root_velocity_w"].astype(f32)], axis=1)
    # compute_reference_trajectory (:213-257)
    vb = cmd["desired_velocity_b"].astype(f32)
    wz = cmd["desired_angular_velocity_b"][:, 2].astype(f32)
    h = cmd["desired_height"].astype(f32)
    dt = params["dt_mpc"].astype(f32)
    c = f32(params["step_dt"])
    tb = dt[:, None] * np.arange(N, dtype=f32)[None, :]  # :218
    wpd[:, 0] = wpd[:, 0] + c * vb[:, 0]
    wpd[:, 1] = wpd[:, 1] + c * vb[:, 1]
    wpd[:, 2] = h
    yaw = yaw + c * wz
    stat = np.abs(vb[:, 0]) < f32(1e-2)
    vw = np.stack([_dot3(Rm[:, i, 0], Rm[:, i, 1], Rm[:, i, 2], vb[:, 0], vb[:, 1], vb[:, 2])
                   for i in range(3)], axis=1)
    xr = np.zeros((B, N, 12), f32)
    xr[:, :, 2] = yaw[:, None] + wz[:, None] * tb
    px = np.where(stat, wpd[:, 0], rp[:, 0])
    py = np.where(stat, wpd[:, 1], rp[:, 1])
    xr[:, :, 3] = px[:, None] + vw[:, 0:1] * tb
    xr[:, :, 4] = py[:, None] + vw[:, 1:2] * tb
    xr[:, :, 5] = h[:, None]
    xr[:, :, 8] = wz[:, None]
    xr[:, :, 9] = vw[:, 0:1]
    xr[:, :, 10] = vw[:, 1:2]
    # input assembly (mpc_controller_cusadi.py:54-95)
    Rflat = Rm.reshape(B, 9) if literal else np.swapaxes(Rm, 1, 2).reshape(B, 9)
    Ib = np.asarray(params["I_body"], f32)
    T = np.stack([np.stack([_dot3(Rm[:, i, 0], Rm[:, i, 1], Rm[:, i, 2], Ib[0, j], Ib[1, j], Ib[2, j])
                            for j in range(3)], 1) for i in range(3)], 1)
    Iw = np.stack([np.stack([_dot3(T[:, i, 0], T[:, i, 1], T[:, i, 2], Rm[:, j, 0], Rm[:, j, 1], Rm[:, j, 2])
                             for j in range(3)], 1) for i in range(3)], 1)
    if gait is not None:
        tab = mpc_gait(gait[0], gait[1], gait[2], N).astype(f32)
    else:
        tab = np.asarray(contact_table, f32)
    ct = tab.reshape(B, 2 * N) if literal else np.swapaxes(tab, 1, 2).reshape(B, 2 * N)
    Q = np.asarray(params["Q"], f32)
    if literal and Q.shape[0] == 13:  # (B,13) tensor read with stride 12
        Qb = np.tile(Q, B)[: 12 * B].reshape(B, 12)
    else:
        Qb = np.tile(Q[:12], (B, 1))
    R = np.tile(np.asarray(params["R"], f32), (B, 1))
    d64 = np.float64
    ins = [x0, np.ones((B, 12 * N)), np.ones((B, 12 * N)), xr.reshape(B, 12 * N), dt[:, None],
           np.full((B, 1), params["mass"], d64), np.full((B, 1), params["mu"], d64), Rflat,
           Iw.reshape(B, 9), rp, st["foot_position"][:, 0, :].astype(f32),
           st["foot_position"][:, 1, :].astype(f32), ct, Qb, R,
           params["residual_lin_accel"].astype(f32), params["residual_ang_accel"].astype(f32)]
    ins = [np.ascontiguousarray(a, d64) for a in ins]
    return ins, {"world_position_desired": wpd, "yaw_desired": yaw, "first_run": fr}


def u0_wrench(N, x, rotation_body):
    """mpc_controller_cusadi.py:186-203: (B, 2, 6) float32 body-frame wrench from u0."""
    u = x[:, 12 * N:12 * N + 12].astype(f32)
    u[:, 6] = 0.0
    u[:, 9] = 0.0
    Rm = rotation_body.astype(f32)
    out = []
    for src in (0, 6, 3, 9):  # left force, left moment, right force, right moment
        v = u[:, src:src + 3]
        out.append(-np.stack([_dot3(Rm[:, 0, i], Rm[:, 1, i], Rm[:, 2, i], v[:, 0], v[:, 1], v[:, 2])
                              for i in range(3)], axis=1))
    return np.concatenate(out, axis=1).reshape(-1, 2, 6)


def stance_torque(wrench, J, contact_bool):
    """leg_controller.py:87-95: tau[b,l] = J[b,l]^T wrench[b,l] where contact_bool[b,l] != 0, else 0.
    float32, the 6-term sum in index order with one rounding per op (as the kernel)."""
    w = wrench.astype(f32)
    J = J.astype(f32)
    t = J[:, :, 0, :] * w[:, :, 0:1]
    for j in range(1, 6):
        t = (t + J[:, :, j, :] * w[:, :, j:j + 1]).astype(f32)
    return np.where(contact_bool[:, :, None] != 0, t, f32(0.0)).astype(f32)
