"""ctypes binding of libsrbd_mpc.so (include/srbd_mpc.h).

The HIP library is the only compute path: if it is missing this module raises; there is no CPU
or PyTorch fallback for the kernels.
"""
from __future__ import annotations

import ctypes
import os

from biped_pympc_amd.build import LIB_DIR

_LIB_NAME = "libsrbd_mpc.so"
_lib = None

_c_dp = ctypes.c_void_p  # device pointers travel as void*


class NativeLibraryMissing(RuntimeError):
    pass


def lib_path() -> str:
    # SRBD_LIB may point at a diagnostic build (scripts/phase_profile.py); default: the product lib
    return os.environ.get("SRBD_LIB") or os.path.join(LIB_DIR, _LIB_NAME)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} not found: build it with `python -m biped_pympc_amd.build` (hipcc, gfx950). "
            "There is no CPU fallback for the SRBD-MPC kernels.")
    L = ctypes.CDLL(path)
    if os.environ.get("SRBD_LIB"):  # an earlier build (A/B runs): bind what it exports
        L = _Tolerant(L)
    L.srbd_abi_version.restype = ctypes.c_int
    L.srbd_last_error.restype = ctypes.c_char_p
    L.srbd_build_id.restype = ctypes.c_char_p
    L.srbd_solver_lds_bytes.restype = ctypes.c_size_t
    L.srbd_solver_lds_bytes.argtypes = [ctypes.c_int]
    L.srbd_mpc_workspace_doubles.restype = ctypes.c_size_t
    L.srbd_mpc_workspace_doubles.argtypes = [ctypes.c_int, ctypes.c_int]
    P = ctypes.POINTER(_c_dp)
    L.srbd_qp_former.restype = ctypes.c_int
    L.srbd_qp_former.argtypes = [ctypes.c_int, ctypes.c_int, P, P, ctypes.c_void_p]
    L.srbd_pdipm.restype = ctypes.c_int
    L.srbd_pdipm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_void_p]
    L.srbd_pdipm_cold.restype = ctypes.c_int
    L.srbd_pdipm_cold.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, P, P,
                                  ctypes.c_void_p]
    L.srbd_pdipm_ccs.restype = ctypes.c_int
    L.srbd_pdipm_ccs.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_void_p]
    L.srbd_mpc_solve.restype = ctypes.c_int
    L.srbd_mpc_solve.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, P,
                                 ctypes.c_void_p, P, ctypes.c_void_p]
    L.srbd_mpc_solve_fused.restype = ctypes.c_int
    L.srbd_mpc_solve_fused.argtypes = L.srbd_mpc_solve.argtypes
    L.srbd_mpc_solve_fused_ex.restype = ctypes.c_int
    L.srbd_mpc_solve_fused_ex.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, P,
                                          ctypes.c_void_p, P, _c_dp, ctypes.c_void_p]
    L.srbd_pdipm_ex.restype = ctypes.c_int
    L.srbd_pdipm_ex.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, P, P,
                                _c_dp, ctypes.c_void_p]
    L.srbd_prepare_device.restype = ctypes.c_int
    L.srbd_prepare_device.argtypes = []
    L.srbd_release_device.restype = ctypes.c_int
    L.srbd_release_device.argtypes = []
    L.srbd_set_scratch_slots.restype = ctypes.c_int
    L.srbd_set_scratch_slots.argtypes = [ctypes.c_int]
    L.srbd_scratch_pool_bytes.restype = ctypes.c_size_t
    L.srbd_scratch_pool_bytes.argtypes = []
    L.srbd_scratch_pool_slots.restype = ctypes.c_int
    L.srbd_scratch_pool_slots.argtypes = []
    L.srbd_scratch_slot_bytes.restype = ctypes.c_size_t
    L.srbd_scratch_slot_bytes.argtypes = []
    L.srbd_evaluate_qp_former.restype = ctypes.c_float
    L.srbd_evaluate_qp_former.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_int]
    L.srbd_evaluate_pdipm.restype = ctypes.c_float
    L.srbd_evaluate_pdipm.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int]
    L.srbd_set_solver_path.restype = ctypes.c_int
    L.srbd_set_solver_path.argtypes = [ctypes.c_int]
    L.srbd_get_solver_path.restype = ctypes.c_int
    L.srbd_get_solver_path.argtypes = []
    L.srbd_set_refinement.restype = ctypes.c_int
    L.srbd_set_refinement.argtypes = [ctypes.c_int]
    L.srbd_get_refinement.restype = ctypes.c_int
    L.srbd_get_refinement.argtypes = []
    L.srbd_set_refinement_policy.restype = ctypes.c_int
    L.srbd_set_refinement_policy.argtypes = [ctypes.c_int, ctypes.c_double]
    L.srbd_pattern_ccs.restype = ctypes.c_int
    L.srbd_pattern_ccs.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                   ctypes.POINTER(ctypes.c_int)]
    L.srbd_prepare_inputs.restype = ctypes.c_int
    L.srbd_prepare_inputs.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(MPCPrep), P, ctypes.c_void_p]
    L.srbd_mpc_step.restype = ctypes.c_int
    L.srbd_mpc_step.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.POINTER(MPCPrep),
                                P, P, _c_dp, ctypes.c_int, _c_dp, _c_dp, _c_dp, ctypes.c_void_p]
    L.srbd_mpc_step_ex.restype = ctypes.c_int
    L.srbd_mpc_step_ex.argtypes = L.srbd_mpc_step.argtypes[:-1] + [_c_dp, ctypes.c_void_p]
    L.srbd_u0_wrench.restype = ctypes.c_int
    L.srbd_u0_wrench.argtypes = [ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp, ctypes.c_void_p]
    L.srbd_u0_wrench_torque.restype = ctypes.c_int
    L.srbd_u0_wrench_torque.argtypes = [ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp, ctypes.c_int, _c_dp,
                                        _c_dp, _c_dp, ctypes.c_void_p]
    L.srbd_dense_scatter.restype = ctypes.c_int
    L.srbd_dense_scatter.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp,
                                     ctypes.c_void_p]
    _lib = L
    return L


class _Tolerant:
    """A library handle whose missing symbols bind to a stub raising on call (SRBD_LIB pointing at a
    build from an earlier tree, for scripts/ab_bench.sh)."""

    class _Missing:
        def __init__(self, name):
            self.name = name

        def __call__(self, *a):
            raise NativeLibraryMissing(f"{self.name} is not exported by {lib_path()}")

    def __init__(self, L):
        object.__setattr__(self, "_L", L)

    def __getattr__(self, name):
        try:
            return getattr(self._L, name)
        except AttributeError:
            stub = _Tolerant._Missing(name)
            object.__setattr__(self, name, stub)
            return stub


class MPCPrep(ctypes.Structure):
    """ctypes mirror of ``srbd_mpc_prep`` (include/srbd_mpc.h); device pointers as void*."""
    _fields_ = [(n, _c_dp) for n in (
        "root_euler", "root_position", "root_angular_velocity_w", "root_velocity_w", "rotation_body",
        "foot_position", "desired_velocity_b", "desired_angular_velocity_b", "desired_height",
        "world_position_desired", "yaw_desired", "first_run", "gait_phase", "ssp_durations",
        "dsp_durations", "contact_table", "dt_mpc", "residual_lin_accel", "residual_ang_accel")] + [
        ("I_body", ctypes.c_float * 9), ("mass", ctypes.c_double), ("mu", ctypes.c_double),
        ("Q", ctypes.c_float * 13), ("q_len", ctypes.c_int), ("R", ctypes.c_float * 12),
        ("step_dt", ctypes.c_float), ("literal_layout", ctypes.c_int)]


def ptr_array(ptrs) -> ctypes.Array:
    arr_t = _c_dp * len(ptrs)
    return arr_t(*[int(p) if p else None for p in ptrs])


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().srbd_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed: {msg}")


SOLVER_PATHS = {"auto": 0, "general": 1, "lds": 2}

# per-problem status word bits (include/srbd_mpc.h SRBD_STATUS_*)
STATUS_NONFINITE, STATUS_STEP_FLOOR, STATUS_FALLBACK = 1, 2, 4


def current_solver_path() -> int:
    """Solver path code in effect for the current HIP device (0 = auto)."""
    return lib().srbd_get_solver_path()


class solver_path:
    """Context manager selecting the solver kernels: "auto" (stage-invariant kernels -- the
    register-resident ones at N = 2..32, the LDS-resident one at N = 1 -- plus the in-launch general
    fallback for a QP that is not stage-invariant), "general" (general kernel only) or "lds" (the
    LDS-resident stage-invariant kernel at every horizon). For the HIP device current on entry; on exit
    the previous path of that device is restored. For tests/benchmarks. ``srbd_mpc_step`` (the
    one-launch controller step) ignores the path."""

    def __init__(self, path: str):
        self.code = SOLVER_PATHS[path]
        self._prev = None
        self._device = None

    def __enter__(self):
        import torch
        self._device = torch.cuda.current_device()
        self._prev = current_solver_path()
        check(lib().srbd_set_solver_path(self.code), "srbd_set_solver_path")
        return self

    def __exit__(self, *exc):
        import torch
        with torch.cuda.device(self._device):
            check(lib().srbd_set_solver_path(self._prev), "srbd_set_solver_path")


REFINEMENT_MODES = {"adaptive": 0, "every_iteration": 1}


def current_refinement() -> int:
    """Affine-refinement mode in effect for the current HIP device (0 = adaptive, the default)."""
    return lib().srbd_get_refinement()


class refinement:
    """Context manager selecting the register kernels' affine-direction refinement (srbd_set_refinement):
    "adaptive" (default: iterations with an ill-conditioned iterate) or "every_iteration" (closer to the
    FP64 floor of the reference's elimination, ~15 % slower at N = 10). For the HIP device
    current on entry; the previous mode of that device is restored on exit."""

    def __init__(self, mode: str):
        self.code = REFINEMENT_MODES[mode]
        self._prev = None
        self._device = None

    def __enter__(self):
        import torch
        self._device = torch.cuda.current_device()
        self._prev = current_refinement()
        check(lib().srbd_set_refinement(self.code), "srbd_set_refinement")
        return self

    def __exit__(self, *exc):
        import torch
        with torch.cuda.device(self._device):  # (an explicit policy before: back to mode 0)
            check(lib().srbd_set_refinement(self._prev if self._prev in (0, 1) else 0), "srbd_set_refinement")


# srbd_set_refinement_policy's word (include/srbd_mpc.h SRBD_REFINE_*)
REFINE_AFFINE_ALL = 1
REFINE_AFFINE_AT_INIT = 2  # at an iterate whose duals are all 1 (a solve's initial iterate)


def refine_affine_first(k: int) -> int:
    return (int(k) & 255) << 8


def refine_affine_last(k: int) -> int:
    return (int(k) & 255) << 16


class refinement_policy:
    """Context manager setting an explicit refinement policy (srbd_set_refinement_policy(flags, w)) on the
    current HIP device -- diagnostics and A/B campaigns (scripts/parity_fuzz.py); on exit the previous
    mode is restored (a previous explicit policy is not: it returns to its mode 0 / 1 default)."""

    def __init__(self, flags: int, w: float = 1e3):
        self.flags, self.w = int(flags), float(w)
        self._prev = None
        self._device = None

    def __enter__(self):
        import torch
        self._device = torch.cuda.current_device()
        self._prev = current_refinement()
        check(lib().srbd_set_refinement_policy(self.flags, self.w), "srbd_set_refinement_policy")
        return self

    def __exit__(self, *exc):
        import torch
        with torch.cuda.device(self._device):
            check(lib().srbd_set_refinement(self._prev if self._prev in (0, 1) else 0), "srbd_set_refinement")


def build_id() -> str:
    """Source hash the loaded libsrbd_mpc.so was built from (build.py source_hash)."""
    try:
        return lib().srbd_build_id().decode()
    except NativeLibraryMissing:
        return "unknown"


def prepare_device() -> None:
    """srbd_prepare_device() on the current HIP device: allocate the solver's per-device pool now.
    Call it before capturing a solver call in a HIP graph (the first solver call on a device
    allocates it otherwise, which a capture does not allow)."""
    check(lib().srbd_prepare_device(), "srbd_prepare_device")


def release_device() -> None:
    """srbd_release_device(): free the current device's pool (device synchronised first)."""
    check(lib().srbd_release_device(), "srbd_release_device")


def set_scratch_slots(slots: int) -> None:
    """srbd_set_scratch_slots(slots): cap the current device's pool (0 = one slot per resident
    workgroup, the default)."""
    check(lib().srbd_set_scratch_slots(int(slots)), "srbd_set_scratch_slots")


def scratch_pool() -> dict:
    """The current device's pool: {"slots", "bytes"} (0 / 0 before it is allocated)."""
    return {"slots": int(lib().srbd_scratch_pool_slots()), "bytes": int(lib().srbd_scratch_pool_bytes())}


def last_error() -> str:
    return lib().srbd_last_error().decode(errors="replace")
