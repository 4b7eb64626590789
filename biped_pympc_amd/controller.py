"""Batched convex-MPC controller over the HIP path -- the caller side of the hot path.

Mirrors the reference controller API so a user of ``MPCControllerCusadi`` can switch:
  * ``MPCConf`` (reference ``biped_pympc/configuration/configuration.py:23-70``),
  * ``StateEStimatorData`` / ``DesiredStateData`` (``biped_pympc/core/data/robot_data.py:9-60``),
  * ``BaseMPCController`` setters and knot-point state (``convex_mpc/base_controller.py:11-266``),
  * ``MPCControllerHIP.run() -> (foot_wrench (B,2,6) float32, cost (B,))`` with the semantics of
    ``MPCControllerCusadi.run`` (``convex_mpc/mpc_controller_cusadi.py:43-205``).
At every horizon the whole step is ONE kernel launch on the caller's current HIP stream with no
host synchronisation (``srbd_mpc_step``): the input preparation (knot points, initial state,
reference trajectory, contact schedule, I_world -- the ~40 small FP32 torch ops of the reference)
into on-chip memory, the fused former + PDIPM (cold start, ``cfg.pdipm_iterations`` Newton
iterations; the reference runs a former call and 4 solver calls x 5 iterations with host round
trips) and the u0 -> wrench (-> stance torque) epilogue; only the (B, 2, 6) wrench leaves the chip
unless ``cfg.keep_solution``. ``run_three_kernel`` runs the same three stages as three kernels
(bit-identical). ``GraphedMPCStep`` replays the step as a captured HIP graph. Nothing of the step is computed in PyTorch; it only owns the buffers.

``literal_layout=True`` (default) reproduces the reference GPU caller's flattening quirks
(row-major R_body read column-major, row-major contact table read column-major, a 13-wide Q read
with stride 12: SURVEY.md Appendix B.1-B.3) so results match the reference; ``False`` lays the
inputs out the way the QP model means them.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Tuple, Union

import torch

from biped_pympc_amd import _native, solver
from biped_pympc_amd.layout import Dims

# robot constants (reference core/robot/hector.py:33-38, core/robot/t1.py:70-75)
ROBOTS = {
    "HECTOR": {"mass": 13.856, "mu": 1.0, "I_body": ((0.5413, 0.0, 0.0), (0.0, 0.5200, 0.0), (0.0, 0.0, 0.0691))},
    "T1": {"mass": 40.0, "mu": 1.0, "I_body": ((0.5413, 0.0, 0.0), (0.0, 0.5200, 0.0), (0.0, 0.0, 0.0691))},
}


@dataclass
class MPCConf:
    """MPC configuration (configuration.py:23-57), plus the HIP path's own knobs."""
    dt: float = 0.001
    dt_mpc: float = 0.025
    horizon_length: int = 10
    decimation: int = 10
    Q: torch.Tensor = field(default_factory=lambda: torch.tensor(
        [150, 150, 250, 100, 100, 250, 1, 1, 5, 10, 10, 1, 1], dtype=torch.float32))
    R: torch.Tensor = field(default_factory=lambda: torch.tensor(
        [1e-5, 1e-5, 1e-5, 1e-5, 1e-5, 1e-5, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4], dtype=torch.float32))
    print_solve_time: bool = False
    solver: str = "hip"
    robot: str = "HECTOR"
    pdipm_iterations: int = 20  # the reference GPU caller: 4 calls x 5 iterations (:28, :144)
    y0: float = 1.0             # dual init of the GPU caller (:141)
    literal_layout: bool = True
    keep_solution: bool = False  # also write the QP solution (x, s, z, y, residuals, mu) to .solution
    #                              and the 17 prepared former inputs to .former_inputs


@dataclass
class StateEStimatorData:
    """Robot state estimate (robot_data.py:9-26), float32, world frame unless noted."""
    num_legs: int = 2
    batch_size: int = 1
    device: Union[torch.device, str] = "cpu"

    def __post_init__(self):
        B, dev = self.batch_size, self.device
        self.root_position = torch.zeros((B, 3), device=dev)
        self.root_quat = torch.zeros((B, 4), device=dev)
        self.root_quat[:, 0] = 1.0
        self.root_euler = torch.zeros((B, 3), device=dev)
        self.rotation_body = torch.eye(3, device=dev).unsqueeze(0).repeat(B, 1, 1)
        self.root_velocity_w = torch.zeros((B, 3), device=dev)
        self.root_angular_velocity_w = torch.zeros((B, 3), device=dev)
        self.foot_position = torch.zeros((B, self.num_legs, 3), device=dev)
        self.root_velocity_b = torch.zeros((B, 3), device=dev)
        self.root_angular_velocity_b = torch.zeros((B, 3), device=dev)


@dataclass
class DesiredStateData:
    """Commanded motion in the body frame (robot_data.py:41-60)."""
    batch_size: int = 1
    device: Union[torch.device, str] = "cpu"

    def __post_init__(self):
        B, dev = self.batch_size, self.device
        self.desired_velocity_b = torch.zeros((B, 3), device=dev)
        self.desired_angular_velocity_b = torch.zeros((B, 3), device=dev)
        self.desired_height = 0.55 * torch.ones(B, device=dev)
        self.desired_position = torch.zeros((B, 3), device=dev)
        self.desired_angle = torch.zeros((B, 3), device=dev)

    def set_command(self, desired_lin_velocity, desired_ang_velocity, desired_height) -> None:
        self.desired_velocity_b[:, :2] = desired_lin_velocity
        self.desired_angular_velocity_b[:, 2] = desired_ang_velocity
        self.desired_height[:] = desired_height


def _f32(t: torch.Tensor, device) -> torch.Tensor:
    return t.to(device=device, dtype=torch.float32).contiguous()


class BaseMPCController:
    """Knot-point state, setters and buffers shared by MPC controllers (base_controller.py:11-266)."""

    def __init__(self, num_envs: int, device: Union[torch.device, str], num_legs: int, cfg: MPCConf):
        self.cfg = cfg
        self.num_envs = num_envs
        self.num_legs = num_legs
        self.device = torch.device(device)
        self.horizon_length = cfg.horizon_length
        self.dt = cfg.dt
        self.dt_mpc = cfg.dt_mpc * torch.ones(num_envs, device=self.device)
        self.state_estimate_data: StateEStimatorData | None = None
        self.desired_state_data: DesiredStateData | None = None
        self.leg_controller_data = None
        self.first_run = torch.ones(num_envs, device=self.device, dtype=torch.bool)
        self._version = 0  # bumped by every setter that replaces a tensor (GraphedMPCStep checks it)
        robot = ROBOTS[cfg.robot]
        self.mass, self.mu = robot["mass"], robot["mu"]
        self.I_body = torch.tensor(robot["I_body"], dtype=torch.float32)
        self.init_buffer()
        self.init_solver()

    def init_buffer(self) -> None:
        B, N, dev = self.num_envs, self.horizon_length, self.device
        self.contact_table = torch.ones((B, N, 2), device=dev)
        self.world_position_desired = torch.zeros((B, 3), device=dev)
        self.yaw_desired = torch.zeros(B, device=dev)
        self.residual_lin_accel = torch.zeros((B, 3), device=dev)
        self.residual_ang_accel = torch.zeros((B, 3), device=dev)
        self.Q = self.cfg.Q
        self.R = self.cfg.R
        self._gait = None  # (phase (B,), ssp (B,2) int32, dsp (B,2) int32) for the device-side schedule

    def init_solver(self) -> None:
        raise NotImplementedError

    # ---- setters (base_controller.py:98-142) ----
    def set_state_estimate_data(self, state_estimate_data: StateEStimatorData) -> None:
        self.state_estimate_data = state_estimate_data
        self._version += 1

    def set_desired_state_data(self, desired_state_data: DesiredStateData) -> None:
        self.desired_state_data = desired_state_data
        self._version += 1

    def set_leg_controller_data(self, leg_controller_data) -> None:
        self.leg_controller_data = leg_controller_data

    def set_contact_table(self, contact_table: torch.Tensor) -> None:
        """Explicit (B, N, 2) contact schedule (what GaitGenerator.mpc_gait returns)."""
        self.contact_table = _f32(contact_table, self.device)
        self._gait = None
        self._version += 1

    def set_gait(self, gait_phase: torch.Tensor, ssp_durations: torch.Tensor, dsp_durations: torch.Tensor) -> None:
        """Device-side contact schedule: the kernel evaluates GaitGenerator.mpc_gait
        (gait_generator.py:216-252) from the phase and SSP/DSP durations at every run()."""
        self._gait = (_f32(gait_phase, self.device),
                      ssp_durations.to(device=self.device, dtype=torch.int32).contiguous(),
                      dsp_durations.to(device=self.device, dtype=torch.int32).contiguous())
        self._version += 1

    def set_mpc_sampling_time(self, dt_mpc: torch.Tensor) -> None:
        self.dt_mpc = dt_mpc
        self._version += 1

    def reset(self, env_ids: torch.Tensor) -> None:
        self.first_run[env_ids] = True


class MPCControllerHIP(BaseMPCController):
    """Drop-in for MPCControllerCusadi: same construction and run() contract, HIP kernels only."""

    def init_solver(self):
        N, B, dev = self.horizon_length, self.num_envs, self.device
        d = Dims(N)
        self.former_inputs = [torch.empty((B, w), dtype=torch.float64, device=dev) for w in d.former_in_nnz]
        self.buffers = solver.MPCSolveBuffers.allocate(N, B, dev)
        self.foot_wrench = torch.empty((B, 2, 6), dtype=torch.float32, device=dev)
        self.cost = torch.zeros(B, device=dev)
        self.tau = None  # (B, 2, ndof) float32, allocated by run_with_torque
        # per-env status word of the last step (include/srbd_mpc.h SRBD_STATUS_*: 1 non-finite
        # solution, 2 step length at its floor in the last iteration): set to an int32 (B,) tensor
        # on the device to have run() fill it (None: not computed)
        self.status = None
        return self

    def _prep_struct(self, keep: list, strict: bool = False) -> _native.MPCPrep:
        """The device-pointer struct of one step. strict (graph capture): every tensor must already
        be float32, contiguous and on the controller's device -- a converted copy would be baked
        into the graph and never see the caller's in-place updates."""
        st, ds, dev = self.state_estimate_data, self.desired_state_data, self.device
        if st is None or ds is None:
            raise RuntimeError("set_state_estimate_data / set_desired_state_data before run()")

        def f32(t, name):
            on_dev = t.device.type == dev.type and (dev.index is None or t.device.index == dev.index)
            if strict and (t.dtype != torch.float32 or not t.is_contiguous() or not on_dev):
                raise ValueError(f"GraphedMPCStep: {name} must be a contiguous float32 tensor on {dev} "
                                 f"(got {t.dtype}, contiguous={t.is_contiguous()}, {t.device})")
            return _f32(t, dev)

        def ptr(t):
            keep.append(t)
            return t.data_ptr()

        p = _native.MPCPrep()
        for name in ("root_euler", "root_position", "root_angular_velocity_w", "root_velocity_w",
                     "rotation_body", "foot_position"):
            setattr(p, name, ptr(f32(getattr(st, name), name)))
        for name in ("desired_velocity_b", "desired_angular_velocity_b", "desired_height"):
            setattr(p, name, ptr(f32(getattr(ds, name), name)))
        for name in ("world_position_desired", "yaw_desired"):  # updated in place by the kernel
            t = getattr(self, name)
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev:
                setattr(self, name, _f32(t, dev))
        if self.first_run.dtype != torch.bool or not self.first_run.is_contiguous():
            self.first_run = self.first_run.to(device=dev, dtype=torch.bool).contiguous()
        p.world_position_desired = ptr(self.world_position_desired)
        p.yaw_desired = ptr(self.yaw_desired)
        p.first_run = ptr(self.first_run)
        if self._gait is not None:
            p.gait_phase, p.ssp_durations, p.dsp_durations = (ptr(t) for t in self._gait)
        else:
            p.contact_table = ptr(f32(self.contact_table, "contact_table"))
        p.dt_mpc = ptr(f32(self.dt_mpc, "dt_mpc"))
        p.residual_lin_accel = ptr(f32(self.residual_lin_accel, "residual_lin_accel"))
        p.residual_ang_accel = ptr(f32(self.residual_ang_accel, "residual_ang_accel"))
        p.I_body[:] = [float(v) for v in self.I_body.reshape(-1).tolist()]
        p.mass, p.mu = float(self.mass), float(self.mu)
        q = [float(v) for v in torch.as_tensor(self.Q, dtype=torch.float32).reshape(-1).tolist()]
        if len(q) not in (12, 13):
            raise ValueError("Q must have 12 (or the reference config's 13) entries")
        p.Q[:len(q)] = q
        p.q_len = len(q)
        p.R[:] = [float(v) for v in torch.as_tensor(self.R, dtype=torch.float32).reshape(-1).tolist()]
        # torch evaluates `decimation * dt * tensor` with the Python product cast to float32
        p.step_dt = float(torch.tensor(self.cfg.decimation * self.cfg.dt, dtype=torch.float32))
        p.literal_layout = 1 if self.cfg.literal_layout else 0
        return p

    def prepare(self) -> list[torch.Tensor]:
        """Write the 17 qp_former inputs for this step (and advance the knot-point state)."""
        keep: list = []
        p = self._prep_struct(keep)
        rc = _native.lib().srbd_prepare_inputs(
            self.horizon_length, self.num_envs, ctypes.byref(p),
            _native.ptr_array([t.data_ptr() for t in self.former_inputs]), solver._stream_ptr())
        _native.check(rc, "srbd_prepare_inputs")
        return self.former_inputs

    def _step(self, p: _native.MPCPrep, J: torch.Tensor | None, cb: torch.Tensor | None) -> None:
        """One srbd_mpc_step launch: prep -> fused former + PDIPM -> wrench (-> torque)."""
        N, B = self.horizon_length, self.num_envs
        outs = (_native.ptr_array([t.data_ptr() for t in self.buffers.outputs])
                if self.cfg.keep_solution else None)
        fin = (_native.ptr_array([t.data_ptr() for t in self.former_inputs])
               if self.cfg.keep_solution else None)
        args = (N, self.cfg.pdipm_iterations, B, float(self.cfg.y0), ctypes.byref(p), fin, outs,
                self.foot_wrench.data_ptr(), 0 if J is None else J.shape[3], None if J is None else J.data_ptr(),
                None if cb is None else cb.data_ptr(), None if J is None else self.tau.data_ptr())
        if self.status is not None:
            rc = _native.lib().srbd_mpc_step_ex(*args, solver._check_status(self.status, B, "MPCControllerHIP.status"),
                                                solver._stream_ptr())
        else:
            rc = _native.lib().srbd_mpc_step(*args, solver._stream_ptr())
        _native.check(rc, "srbd_mpc_step")
        self.solution = self.buffers.outputs if self.cfg.keep_solution else None

    def run(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """MPCControllerCusadi.run (mpc_controller_cusadi.py:43-205): (foot_wrench (B,2,6) f32, cost)."""
        keep: list = []
        self._step(self._prep_struct(keep), None, None)
        return self.foot_wrench, self.cost

    def run_three_kernel(self, J: torch.Tensor | None = None, cb: torch.Tensor | None = None):
        """The same step as three launches (srbd_prepare_inputs -> srbd_mpc_solve_fused ->
        srbd_u0_wrench_torque) with the 17 former inputs and the solution in device memory.
        Bit-identical to run() (tests/test_controller.py)."""
        N, B = self.horizon_length, self.num_envs
        self.prepare()
        out = solver.mpc_solve(self.former_inputs, N, self.cfg.pdipm_iterations, self.cfg.y0, self.buffers)
        self.solution = out if self.cfg.keep_solution else None  # as run(): exposed on request only
        rot = _f32(self.state_estimate_data.rotation_body, self.device)
        rc = _native.lib().srbd_u0_wrench_torque(
            N, B, out[0].data_ptr(), rot.data_ptr(), self.foot_wrench.data_ptr(), 0 if J is None else J.shape[3],
            None if J is None else J.data_ptr(), None if cb is None else cb.data_ptr(),
            None if J is None else self.tau.data_ptr(), solver._stream_ptr())
        _native.check(rc, "srbd_u0_wrench_torque")
        return (self.foot_wrench, self.cost) if J is None else (self.foot_wrench, self.cost, self.tau)

    def _torque_args(self, contact_jacobian, contact_bool):
        B = self.num_envs
        J = _f32(contact_jacobian, self.device)
        cb = _f32(contact_bool, self.device)
        if J.dim() != 4 or J.shape[:3] != (B, 2, 6) or cb.shape != (B, 2):
            raise ValueError(f"contact_jacobian must be ({B},2,6,ndof) and contact_bool ({B},2)")
        ndof = J.shape[3]
        if self.tau is None or self.tau.shape != (B, 2, ndof):
            self.tau = torch.empty((B, 2, ndof), dtype=torch.float32, device=self.device)
        return J, cb

    def run_with_torque(self, contact_jacobian: torch.Tensor, contact_bool: torch.Tensor
                        ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """run() plus the stance feed-forward joint torque the wrench feeds
        (LegController.update_ff_torque, leg_controller.py:87-95, after
        BipedController._run_stance_leg_controller, biped_controller.py:144-146), computed in the
        step's epilogue: tau (B,2,ndof) float32 = J[:,l]^T wrench[:,l] on stance legs, 0 on swing
        legs. contact_jacobian (B,2,6,ndof) float32 (LegControllerData.J), contact_bool (B,2)."""
        J, cb = self._torque_args(contact_jacobian, contact_bool)
        keep: list = []
        self._step(self._prep_struct(keep), J, cb)
        return self.foot_wrench, self.cost, self.tau


# the reference's class name, for drop-in imports
MPCControllerCusadi = MPCControllerHIP


class GraphedMPCStep:
    """The controller step captured once as a HIP graph and replayed (one graph launch per step; the
    graph holds the single srbd_mpc_step kernel). Worth it when the batch is
    small and launch overhead is a visible share of the step.

    The graph records device pointers, so the state / command / schedule tensors must be contiguous
    float32 on the controller's device at capture (checked) and be updated IN PLACE (``copy_``)
    between replays. Every replay first compares the storage of every source tensor -- the state
    estimate and command fields, the contact schedule, dt_mpc, the residual accelerations, the
    knot-point state -- with what was captured, and the constants baked into the graph (mass, mu,
    I_body, Q, R, step dt, layout, iterations, y0, the device's refinement mode of srbd_set_refinement):
    a tensor replaced by assignment
    (``data.root_position = ...``, ``c.residual_lin_accel = x.clone()``, a setter) or a changed
    constant makes the replay raise instead of silently reading the captured values. (Q and R given
    as device tensors are compared by storage, not value.)
    """

    def __init__(self, controller: MPCControllerHIP, warmup: int = 1):
        self.c = controller
        self._keep: list = []
        self._prep = self.c._prep_struct(self._keep, strict=True)  # resolves every input pointer once
        self._version = controller._version
        self._signature = self._current_signature()
        saved = [t.clone() for t in (controller.world_position_desired, controller.yaw_desired,
                                     controller.first_run)]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):  # first launches configure kernel attributes outside capture
                self._launch()
        torch.cuda.current_stream().wait_stream(s)
        for dst, src in zip((controller.world_position_desired, controller.yaw_desired,
                             controller.first_run), saved):
            dst.copy_(src)  # the warm-up must not advance the knot-point state
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._launch()

    def _launch(self) -> None:
        self.c._step(self._prep, None, None)

    def _current_signature(self) -> tuple:
        """(name, storage pointer) of every tensor the step reads or updates, plus the constants the
        graph bakes in -- without converting or synchronising anything."""
        c, st, ds = self.c, self.c.state_estimate_data, self.c.desired_state_data
        src = [(n, getattr(st, n)) for n in ("root_euler", "root_position", "root_angular_velocity_w",
                                             "root_velocity_w", "rotation_body", "foot_position")]
        src += [(n, getattr(ds, n)) for n in ("desired_velocity_b", "desired_angular_velocity_b", "desired_height")]
        src += [(n, getattr(c, n)) for n in ("world_position_desired", "yaw_desired", "first_run", "dt_mpc",
                                             "residual_lin_accel", "residual_ang_accel")]
        if c._gait is not None:
            src += list(zip(("gait_phase", "ssp_durations", "dsp_durations"), c._gait))
        else:
            src.append(("contact_table", c.contact_table))

        def value(v):
            if isinstance(v, torch.Tensor):
                return ("device", v.data_ptr()) if v.is_cuda else tuple(v.reshape(-1).tolist())
            return tuple(v) if isinstance(v, (list, tuple)) else v
        consts = (("mass", c.mass), ("mu", c.mu), ("I_body", value(c.I_body)), ("Q", value(c.Q)),
                  ("R", value(c.R)), ("step_dt", c.cfg.decimation * c.cfg.dt),
                  ("literal_layout", c.cfg.literal_layout), ("pdipm_iterations", c.cfg.pdipm_iterations),
                  ("y0", c.cfg.y0), ("keep_solution", c.cfg.keep_solution),
                  ("refinement", _native.current_refinement()))  # baked into the kernel's arguments
        return tuple((n, t.data_ptr()) for n, t in src) + consts

    def __call__(self) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.c._version != self._version:
            raise RuntimeError("GraphedMPCStep: a controller setter replaced a captured tensor since the "
                               "capture; update tensors in place, or capture a new GraphedMPCStep")
        sig = self._current_signature()
        if sig != self._signature:
            changed = [a[0] for a, b in zip(sig, self._signature) if a != b]
            raise RuntimeError(f"GraphedMPCStep: {', '.join(changed)} replaced or changed since the capture "
                               "(the graph would read the captured values); update tensors in place, or "
                               "capture a new GraphedMPCStep")
        self.graph.replay()
        return self.c.foot_wrench, self.c.cost


def dense_scatter(values: torch.Tensor, inverse_index: torch.Tensor, shape: tuple[int, int],
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """(B, nnz) nonzeros -> (B, rows, cols) dense through ``inverse_index`` (int32 (rows*cols,),
    nonzero index or -1) with one scatter kernel (CusadiFunction.getDenseOutput replacement)."""
    B, nnz = values.shape
    rc = shape[0] * shape[1]
    if out is None:
        out = torch.empty((B, shape[0], shape[1]), dtype=torch.float64, device=values.device)
    vals = values.contiguous()
    for lo in range(0, B, 65535):  # grid.y limit per launch
        hi = min(B, lo + 65535)
        rc_ = _native.lib().srbd_dense_scatter(hi - lo, nnz, rc, inverse_index.data_ptr(),
                                               vals[lo:hi].data_ptr(), out[lo:hi].data_ptr(),
                                               solver._stream_ptr())
        _native.check(rc_, "srbd_dense_scatter")
    return out


def inverse_index(rows, cols, shape: tuple[int, int], device) -> torch.Tensor:
    """Dense position -> nonzero index map of a sparsity given as triplets (-1 = structural zero)."""
    inv = torch.full((shape[0] * shape[1],), -1, dtype=torch.int32)
    lin = torch.as_tensor(rows, dtype=torch.int64) * shape[1] + torch.as_tensor(cols, dtype=torch.int64)
    inv[lin] = torch.arange(lin.numel(), dtype=torch.int32)
    return inv.to(device)
