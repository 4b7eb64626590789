"""The MPC step around the QP: input preparation, u0 -> wrench, dense output, the controller.

CPU tests pin the oracle (oracle/mpc_io.py): the contact schedule against tables produced by the
REFERENCE GaitGenerator (tests/golden/gait_reference.npz), and the FP32 restatement against the
same op sequence executed by torch on CPU (the reference's own framework; base_controller.py cannot
be imported here because its package pulls CasADi). GPU tests compare the HIP kernels with the
oracle bit for bit, and the whole controller step (prepare -> former -> 20-iteration PDIPM ->
wrench) with the oracle pipeline.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest
import torch

from oracle import mpc_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


def random_robot(B, seed, N=10, gait=True):
    """Float32 state estimate / command / controller state, SURVEY 8d distributions."""
    from biped_pympc_amd.utils.synthetic import rot_zyx
    rng = np.random.default_rng(seed)
    eul = np.stack([rng.uniform(-0.15, 0.15, B), rng.uniform(-0.15, 0.15, B), rng.uniform(-np.pi, np.pi, B)], 1)
    R = rot_zyx(eul[:, 0], eul[:, 1], eul[:, 2])
    pos = np.stack([rng.uniform(-1, 1, B), rng.uniform(-1, 1, B), 0.55 + rng.uniform(-0.03, 0.03, B)], 1)
    feet = np.stack([pos + np.einsum("bij,j->bi", R, [0.0, 0.10, -0.55]),
                     pos + np.einsum("bij,j->bi", R, [0.0, -0.10, -0.55])], 1)
    vb = np.stack([rng.uniform(-1, 1, B), rng.uniform(-1, 1, B), np.zeros(B)], 1)
    vb[::4, 0] = 0.0  # some stationary envs (|v_x| < 1e-2 branch)
    st = {"root_euler": eul, "root_position": pos, "root_angular_velocity_w": rng.normal(0, 0.2, (B, 3)),
          "root_velocity_w": rng.normal(0, 0.3, (B, 3)), "rotation_body": R, "foot_position": feet}
    cmd = {"desired_velocity_b": vb,
           "desired_angular_velocity_b": np.stack([np.zeros(B), np.zeros(B), rng.uniform(-1, 1, B)], 1),
           "desired_height": 0.55 + rng.uniform(-0.02, 0.02, B)}
    ctrl = {"world_position_desired": rng.normal(0, 0.5, (B, 3)), "yaw_desired": rng.uniform(-1, 1, B),
            "first_run": (np.arange(B) % 3 == 0)}
    params = {"dt_mpc": np.full(B, 0.025) + rng.uniform(0, 0.005, B), "residual_lin_accel": rng.normal(0, 0.3, (B, 3)),
              "residual_ang_accel": rng.normal(0, 0.3, (B, 3)), "I_body": np.diag([0.5413, 0.52, 0.0691]),
              "mass": 13.856, "mu": 1.0,
              "Q": np.array([150, 150, 250, 100, 100, 250, 1, 1, 5, 10, 10, 1, 1], np.float32),
              "R": np.array([1e-5] * 6 + [1e-4] * 6, np.float32), "step_dt": np.float32(10 * 0.001)}
    for dct in (st, cmd, params):
        for k, v in list(dct.items()):
            if isinstance(v, np.ndarray) and v.dtype == np.float64 and k != "I_body":
                dct[k] = v.astype(np.float32)
    gait_args = None
    if gait:
        gait_args = (rng.uniform(0, 1, B).astype(np.float32), rng.integers(3, 7, (B, 2)), rng.integers(0, 3, (B, 2)))
    table = rng.integers(0, 2, (B, N, 2)).astype(np.float32)
    return st, cmd, ctrl, params, gait_args, table


# ------------------------------------------------------------------------------ CPU ----

def test_oracle_gait_matches_reference_module():
    g = np.load(os.path.join(GOLD, "gait_reference.npz"))
    tab = mpc_io.mpc_gait(g["phase"], g["ssp"], g["dsp"], g["table"].shape[1])
    assert np.array_equal(tab, g["table"])


def test_oracle_fp32_semantics_match_torch():
    """The numpy restatement rounds exactly like the reference's torch FP32 op sequence
    (base_controller.py:218-257 executed with torch on CPU, one op at a time)."""
    N, B = 10, 33
    st, cmd, ctrl, params, _, table = random_robot(B, 5, N, gait=False)
    ins, new = mpc_io.prepare_inputs(N, st, cmd, ctrl, params, contact_table=table)
    T = {k: torch.from_numpy(np.asarray(v)) for d in (st, cmd, params) for k, v in d.items()
         if isinstance(v, np.ndarray) and k != "I_body"}
    wpd = torch.from_numpy(ctrl["world_position_desired"].astype(np.float32))
    yaw = torch.from_numpy(ctrl["yaw_desired"].astype(np.float32))
    fr = torch.from_numpy(ctrl["first_run"])
    wpd[fr] = T["root_position"][fr]
    yaw[fr] = T["root_euler"][fr, 2]
    tb = T["dt_mpc"][:, None] * torch.arange(0, N).unsqueeze(0).repeat(B, 1)
    step = 10 * 0.001
    wpd[:, 0] += step * T["desired_velocity_b"][:, 0]
    wpd[:, 1] += step * T["desired_velocity_b"][:, 1]
    wpd[:, 2] = T["desired_height"]
    yaw += step * T["desired_angular_velocity_b"][:, 2]
    xr = torch.zeros(B, N, 12)
    xr[:, :, 2] = yaw.unsqueeze(1) + T["desired_angular_velocity_b"][:, 2].unsqueeze(1) * tb
    xr[:, :, 5] = T["desired_height"].unsqueeze(1).repeat(1, N)
    assert torch.equal(wpd, torch.from_numpy(new["world_position_desired"]))
    assert torch.equal(yaw, torch.from_numpy(new["yaw_desired"]))
    ref = ins[3].reshape(B, N, 12)
    assert np.array_equal(ref[:, :, 2], xr[:, :, 2].double().numpy())
    assert np.array_equal(ref[:, :, 5], xr[:, :, 5].double().numpy())


def test_oracle_literal_q_is_the_strided_read_of_13_weights():
    N, B = 10, 27
    st, cmd, ctrl, params, _, table = random_robot(B, 6, N, gait=False)
    ins, _ = mpc_io.prepare_inputs(N, st, cmd, ctrl, params, contact_table=table, literal=True)
    flat = np.tile(params["Q"], B)  # the caller's (B, 13) tensor, flattened
    for e in (0, 1, 12, 26):
        assert np.array_equal(ins[13][e], flat[12 * e:12 * e + 12].astype(np.float64))
    ins_c, _ = mpc_io.prepare_inputs(N, st, cmd, ctrl, params, contact_table=table, literal=False)
    assert np.array_equal(ins_c[13], np.tile(params["Q"][:12], (B, 1)).astype(np.float64))
    assert np.array_equal(ins_c[7].reshape(B, 3, 3), np.swapaxes(st["rotation_body"], 1, 2).astype(np.float64))


def test_prep_struct_layout_matches_header(tmp_path):
    from biped_pympc_amd import _native
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "srbd_mpc.h"\nint main(){printf("%zu %zu %zu %zu %zu",'
                   "sizeof(srbd_mpc_prep), offsetof(srbd_mpc_prep, I_body), offsetof(srbd_mpc_prep, mass),"
                   "offsetof(srbd_mpc_prep, q_len), offsetof(srbd_mpc_prep, literal_layout));}\n")
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    M = _native.MPCPrep
    assert got == [ctypes.sizeof(M), M.I_body.offset, M.mass.offset, M.q_len.offset, M.literal_layout.offset]


# ------------------------------------------------------------------------------ GPU ----

def _controller(B, N, st, cmd, ctrl, params, gait_args, table, literal=True):
    from biped_pympc_amd.controller import DesiredStateData, MPCConf, MPCControllerHIP, StateEStimatorData
    cfg = MPCConf(horizon_length=N, Q=torch.from_numpy(params["Q"]), R=torch.from_numpy(params["R"]),
                  literal_layout=literal)
    c = MPCControllerHIP(B, "cuda", 2, cfg)
    se = StateEStimatorData(2, B, "cuda")
    for k in ("root_euler", "root_position", "root_angular_velocity_w", "root_velocity_w", "rotation_body",
              "foot_position"):
        setattr(se, k, torch.from_numpy(st[k]).cuda())
    ds = DesiredStateData(B, "cuda")
    for k in ("desired_velocity_b", "desired_angular_velocity_b", "desired_height"):
        setattr(ds, k, torch.from_numpy(cmd[k]).cuda())
    c.set_state_estimate_data(se)
    c.set_desired_state_data(ds)
    c.world_position_desired = torch.from_numpy(ctrl["world_position_desired"].astype(np.float32)).cuda()
    c.yaw_desired = torch.from_numpy(ctrl["yaw_desired"].astype(np.float32)).cuda()
    c.first_run = torch.from_numpy(ctrl["first_run"]).cuda()
    c.set_mpc_sampling_time(torch.from_numpy(params["dt_mpc"]).cuda())
    c.residual_lin_accel = torch.from_numpy(params["residual_lin_accel"]).cuda()
    c.residual_ang_accel = torch.from_numpy(params["residual_ang_accel"]).cuda()
    if gait_args is not None:
        c.set_gait(*(torch.from_numpy(np.asarray(a)) for a in gait_args))
    else:
        c.set_contact_table(torch.from_numpy(table))
    return c


@pytest.mark.gpu
@pytest.mark.parametrize("gait,literal", [(True, True), (False, True), (True, False)])
def test_prepare_inputs_matches_oracle(gait, literal):
    N, B = 10, 300
    st, cmd, ctrl, params, gait_args, table = random_robot(B, 11, N, gait=gait)
    c = _controller(B, N, st, cmd, ctrl, params, gait_args, table, literal)
    got = [t.cpu().numpy() for t in c.prepare()]
    torch.cuda.synchronize()
    ref, new = mpc_io.prepare_inputs(N, st, cmd, ctrl, params, gait=gait_args, contact_table=table, literal=literal)
    for k, (g, r) in enumerate(zip(got, ref)):
        assert np.array_equal(g, r), f"former input {k}: max diff {np.abs(g - r).max():.3e}"
    assert np.array_equal(c.world_position_desired.cpu().numpy(), new["world_position_desired"])
    assert np.array_equal(c.yaw_desired.cpu().numpy(), new["yaw_desired"])
    assert not c.first_run.any()


@pytest.mark.gpu
def test_u0_wrench_matches_oracle():
    from biped_pympc_amd import _native, solver
    N, B = 10, 1000
    rng = np.random.default_rng(3)
    x = rng.normal(0, 50, (B, 24 * N))
    R = np.linalg.qr(rng.normal(size=(B, 3, 3)))[0].astype(np.float32)
    out = torch.empty((B, 2, 6), dtype=torch.float32, device="cuda")
    xd, Rd = torch.from_numpy(x).cuda(), torch.from_numpy(R).cuda()
    _native.check(_native.lib().srbd_u0_wrench(N, B, xd.data_ptr(), Rd.data_ptr(), out.data_ptr(),
                                               solver._stream_ptr()), "wrench")
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), mpc_io.u0_wrench(N, x, R))


def _torque_inputs(B, ndof, seed):
    rng = np.random.default_rng(seed)
    J = rng.normal(0, 0.3, (B, 2, 6, ndof)).astype(np.float32)
    cb = (rng.uniform(size=(B, 2)) < 0.7).astype(np.float32)
    cb[0] = 0.0  # both legs swinging
    cb[1] = 1.0  # double support
    return J, cb


@pytest.mark.parametrize("ndof", [5, 6])
def test_stance_torque_oracle_matches_torch(ndof):
    """The restatement against the reference's own op sequence on torch CPU
    (leg_controller.py:87-95: J^T @ f, then torch.where on the contact flag)."""
    B = 257
    J, cb = _torque_inputs(B, ndof, 4)
    w = np.random.default_rng(5).normal(0, 80, (B, 2, 6)).astype(np.float32)
    Jt, wt, cbt = torch.from_numpy(J), torch.from_numpy(w), torch.from_numpy(cb)
    ref = torch.empty(B, 2, ndof)
    for leg in range(2):
        st = (Jt[:, leg].transpose(1, 2) @ wt[:, leg].unsqueeze(-1)).squeeze(-1)
        ref[:, leg] = torch.where(cbt[:, leg].unsqueeze(-1).bool(), st, torch.zeros_like(st))
    got = mpc_io.stance_torque(w, J, cb)
    assert got.dtype == np.float32
    assert np.all(got[cb == 0] == 0.0)
    # 6-term FP32 dot: the summation order of torch's matmul is implementation-defined
    np.testing.assert_allclose(got, ref.numpy(), rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("ndof", [5, 6])
def test_u0_wrench_torque_matches_oracle(ndof):
    from biped_pympc_amd import _native, solver
    N, B = 10, 1000
    rng = np.random.default_rng(6)
    x = rng.normal(0, 50, (B, 24 * N))
    R = np.linalg.qr(rng.normal(size=(B, 3, 3)))[0].astype(np.float32)
    J, cb = _torque_inputs(B, ndof, 7)
    w = torch.empty((B, 2, 6), dtype=torch.float32, device="cuda")
    tau = torch.full((B, 2, ndof), float("nan"), dtype=torch.float32, device="cuda")
    xd, Rd, Jd, cbd = (torch.from_numpy(a).cuda() for a in (x, R, J, cb))
    _native.check(_native.lib().srbd_u0_wrench_torque(N, B, xd.data_ptr(), Rd.data_ptr(), w.data_ptr(), ndof,
                                                      Jd.data_ptr(), cbd.data_ptr(), tau.data_ptr(),
                                                      solver._stream_ptr()), "wrench+torque")
    torch.cuda.synchronize()
    wref = mpc_io.u0_wrench(N, x, R)
    assert np.array_equal(w.cpu().numpy(), wref)
    assert np.array_equal(tau.cpu().numpy(), mpc_io.stance_torque(wref, J, cb))
    # bad arguments are reported, not aborted on
    assert _native.lib().srbd_u0_wrench_torque(N, B, xd.data_ptr(), Rd.data_ptr(), w.data_ptr(), 0,
                                               Jd.data_ptr(), cbd.data_ptr(), tau.data_ptr(),
                                               solver._stream_ptr()) != 0


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["H", "A", "G"])
def test_dense_scatter_matches_layout(which):
    from biped_pympc_amd import layout
    from biped_pympc_amd.controller import dense_scatter, inverse_index
    N, B = 10, 64
    d = layout.Dims(N)
    cp, ri = {"H": layout.ccs_H, "A": layout.ccs_A, "G": layout.ccs_G}[which](N)
    shape = {"H": (d.nz, d.nz), "A": (d.n_eq, d.nz), "G": (d.n_ineq, d.nz)}[which]
    rows, cols = layout.triplet(cp, ri)
    vals = np.random.default_rng(1).normal(size=(B, len(rows)))
    inv = inverse_index(rows, cols, shape, "cuda")
    dense = dense_scatter(torch.from_numpy(vals).cuda(), inv, shape).cpu().numpy()
    ref = layout.to_dense(vals, cp, ri, shape)
    assert np.array_equal(dense, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("N,K", [(10, 20), (10, 30), (5, 20), (32, 20), (1, 30)])
def test_controller_step_matches_oracle_pipeline(N, K):
    """prepare -> fused former + K-iteration PDIPM -> wrench against the oracle pipeline.

    K = 20 is the controller default (the reference's 4 x 5 schedule). Every env must meet
    north_star's 1e-4 relative wrench error at K = 20 and 1e-6 at K = 30 (converged). The wrench is
    FP32, so errors are relative to max(|wrench|, 1 N).
    """
    from oracle import oracle
    B = 128
    st, cmd, ctrl, params, gait_args, table = random_robot(B, 21, N, gait=True)
    c = _controller(B, N, st, cmd, ctrl, params, gait_args, table)
    c.cfg.pdipm_iterations = K
    wrench, cost = c.run()
    torch.cuda.synchronize()
    ins, _ = mpc_io.prepare_inputs(N, st, cmd, ctrl, params, gait=gait_args)
    x = oracle.mpc_solve(N, K, ins, y0=1.0)[0]
    ref = mpc_io.u0_wrench(N, x, st["rotation_body"])
    w = wrench.cpu().numpy()
    assert w.shape == (B, 2, 6) and w.dtype == np.float32 and cost.shape == (B,)
    rel = lambda a, r: np.abs(a - r).max(axis=(1, 2)) / np.maximum(np.abs(r).max(axis=(1, 2)), 1.0)
    err = rel(w, ref)
    bar = 1e-6 if K >= 30 else 1e-4
    # an env above the bar must sit within 4x of its FP64 floor: the distance between the oracle
    # (sparse LDL^T) and the independent dense-LU restatement of the same solve (one N = 1 env's
    # two CPU solutions differ by 2.4e-4 in the wrench at K = 30)
    from oracle.pdipm_dense import pdipm_dense
    from biped_pympc_amd.utils.synthetic import solver_init
    H, f, A, b, G, d = oracle.qp_former(N, ins)
    it = solver_init(d, N, y0=1.0)
    for e in np.flatnonzero(err > bar):
        xd = pdipm_dense(N, K, H[e], G[e], A[e], f[e], d[e], b[e], *(t[e] for t in it))[0]
        floor = rel(mpc_io.u0_wrench(N, xd[None], st["rotation_body"][e:e + 1]), ref[e:e + 1])[0]
        assert err[e] <= 4.0 * floor, (e, err[e], floor)


@pytest.mark.gpu
def test_controller_run_with_torque():
    N, B, ndof = 10, 64, 5
    st, cmd, ctrl, params, gait_args, table = random_robot(B, 22, N, gait=True)
    J, cb = _torque_inputs(B, ndof, 8)
    c1 = _controller(B, N, st, cmd, ctrl, params, gait_args, table)
    c2 = _controller(B, N, st, cmd, ctrl, params, gait_args, table)
    w1, _ = c1.run()
    w2, _, tau = c2.run_with_torque(torch.from_numpy(J), torch.from_numpy(cb))
    torch.cuda.synchronize()
    assert torch.equal(w1, w2)
    assert tau.shape == (B, 2, ndof)
    assert np.array_equal(tau.cpu().numpy(), mpc_io.stance_torque(w2.cpu().numpy(), J, cb))


@pytest.mark.gpu
@pytest.mark.parametrize("N", [10, 5])
def test_graphed_step_replays_the_controller_step(N):
    """GraphedMPCStep: one captured graph launch per step, same wrench as run(), and replays pick
    up state updated in place (N = 5: the LDS-resident one-launch step)."""
    from biped_pympc_amd.controller import GraphedMPCStep
    B = 64
    st, cmd, ctrl, params, gait_args, table = random_robot(B, 31, N, gait=True)
    c1 = _controller(B, N, st, cmd, ctrl, params, gait_args, table)
    c2 = _controller(B, N, st, cmd, ctrl, params, gait_args, table)
    g = GraphedMPCStep(c2)  # the warm-up launch leaves c2's knot-point state as it was
    for step in range(3):
        w1, _ = c1.run()
        w2, _ = g()
        torch.cuda.synchronize()
        assert torch.equal(w1, w2), step
        # move the robots: in-place updates are seen by the next replay
        for c in (c1, c2):
            c.state_estimate_data.root_position.add_(0.01)
            c.state_estimate_data.foot_position.add_(0.01)


@pytest.mark.gpu
@pytest.mark.parametrize("N,gait,literal,torque", [(10, True, True, False), (10, False, True, True),
                                                   (20, True, False, True), (10, True, True, True),
                                                   (5, True, True, True), (32, False, False, False),
                                                   (1, True, True, False)])
def test_one_launch_step_equals_three_kernels(N, gait, literal, torque):
    """srbd_mpc_step (prep -> fused former + PDIPM -> wrench / torque in ONE kernel, inputs kept
    on chip) against the three-launch sequence it replaces: wrench, torque, solution and the
    advanced knot-point state bit for bit, over three consecutive steps."""
    B, ndof = 77, 6
    st, cmd, ctrl, params, gait_args, table = random_robot(B, 41 + N, N, gait=gait)
    c1 = _controller(B, N, st, cmd, ctrl, params, gait_args, table, literal)
    c2 = _controller(B, N, st, cmd, ctrl, params, gait_args, table, literal)
    c1.cfg.keep_solution = True
    c2.cfg.keep_solution = True
    J, cb = (torch.from_numpy(a) for a in _torque_inputs(B, ndof, 9))
    for step in range(3):
        if torque:
            w1, _, t1 = c1.run_with_torque(J, cb)
            J2, cb2 = c2._torque_args(J, cb)
            w2, _, t2 = c2.run_three_kernel(J2, cb2)
            torch.cuda.synchronize()
        else:
            w1, _ = c1.run()
            w2, _ = c2.run_three_kernel()
            torch.cuda.synchronize()
        for i, (a, b) in enumerate(zip(c1.former_inputs, c2.former_inputs)):
            assert torch.equal(a, b), (step, "former input", i, (a - b).abs().max().item())
        for i, (a, b) in enumerate(zip(c1.solution, c2.solution)):
            assert torch.equal(a, b), (step, "solution", i, (a - b).abs().max().item())
        assert torch.equal(w1, w2), step
        if torque:
            assert torch.equal(t1, t2), step
        for name in ("world_position_desired", "yaw_desired", "first_run"):
            assert torch.equal(getattr(c1, name), getattr(c2, name)), (step, name)


@pytest.mark.gpu
def test_one_launch_step_writes_only_the_wrench():
    """keep_solution False (default): the step's solution buffers are left untouched."""
    N, B = 10, 32
    st, cmd, ctrl, params, gait_args, table = random_robot(B, 51, N, gait=True)
    c = _controller(B, N, st, cmd, ctrl, params, gait_args, table)
    for t in c.buffers.outputs:
        t.fill_(7.0)
    w, _ = c.run()
    torch.cuda.synchronize()
    assert c.solution is None and torch.isfinite(w).all()
    assert all(bool((t == 7.0).all()) for t in c.buffers.outputs)


@pytest.mark.gpu
def test_graphed_step_refuses_stale_or_converted_tensors():
    from biped_pympc_amd.controller import GraphedMPCStep
    N, B = 10, 16
    st, cmd, ctrl, params, gait_args, table = random_robot(B, 61, N, gait=False)
    c = _controller(B, N, st, cmd, ctrl, params, gait_args, table)
    c.state_estimate_data.root_position = c.state_estimate_data.root_position.double()
    with pytest.raises(ValueError, match="root_position"):
        GraphedMPCStep(c)
    c.state_estimate_data.root_position = c.state_estimate_data.root_position.float()
    g = GraphedMPCStep(c)
    g()
    c.set_contact_table(torch.from_numpy(table))  # replaces a captured tensor
    with pytest.raises(RuntimeError, match="replaced"):
        g()
    # direct field assignment, as the reference's StateEstimator.set_body_state and
    # mpc_wrapper.set_srbd_accel do, bypasses the setters: the replay still refuses
    g = GraphedMPCStep(c)
    g()
    c.state_estimate_data.root_position = c.state_estimate_data.root_position.clone()
    with pytest.raises(RuntimeError, match="root_position"):
        g()
    g = GraphedMPCStep(c)
    c.residual_lin_accel = c.residual_lin_accel.clone()
    with pytest.raises(RuntimeError, match="residual_lin_accel"):
        g()
    g = GraphedMPCStep(c)
    c.mass = c.mass * 1.1  # a constant the graph baked in
    with pytest.raises(RuntimeError, match="mass"):
        g()
    c.mass = c.mass / 1.1
    from biped_pympc_amd import _native
    g = GraphedMPCStep(c)
    with _native.refinement("every_iteration"):  # the refinement mode is baked into the kernel's arguments
        with pytest.raises(RuntimeError, match="refinement"):
            g()
    g = GraphedMPCStep(c)
    c.state_estimate_data.root_position.add_(0.01)  # in-place updates stay fine
    g()
