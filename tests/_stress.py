"""Stress workloads for the parity tests (shared by tests/test_gpu_stress.py and the fixture script
tests/golden/make_stress_floor.py): regimes the SURVEY 8d distributions rarely reach."""
import numpy as np

from biped_pympc_amd.utils.synthetic import make_workload

STRESS_B = 24
STRESS_K = (10, 20)


def _contact(B, N, left, right):
    c = np.zeros((B, N, 2), np.int32)
    c[:, :, 0] = left
    c[:, :, 1] = right
    return c


# name -> (N, make_workload keyword arguments)
STRESS_CASES = {
    # both feet in swing over the whole horizon: fz <= fmax * 0 and -fz <= 0 pin every force to 0
    # (all friction-cone rows of a foot active together: degenerate complementarity)
    "flight_N10": (10, dict(contact_override=_contact(STRESS_B, 10, 0, 0))),
    # the left foot in swing throughout, the right one carrying the robot
    "swing_left_N20": (20, dict(contact_override=_contact(STRESS_B, 20, 0, 1))),
    # roll / pitch up to 0.6 rad with a randomized gait and RL residuals
    "tilt_N10": (10, dict(tilt=0.6, random_gait=True, residuals=True)),
    # residual accelerations of std 3 m/s^2 / 3 rad/s^2 (6x the SURVEY spread), randomized gait
    "push_N20": (20, dict(random_gait=True, residuals=True, residual_scale=3.0)),
    # two more horizons (the regN register kernels under the auto path, the runtime-N LDS-resident
    # kernel under "lds"): flight at N = 5, and the right foot in swing over a 32-stage horizon with
    # tilt and residuals
    "flight_N5": (5, dict(contact_override=_contact(STRESS_B, 5, 0, 0))),
    "swing_right_N32": (32, dict(contact_override=_contact(STRESS_B, 32, 1, 0), tilt=0.3, residuals=True)),
}


# fixed seeds (the first four are the round-2 cases' seeds, 9000 + their sorted position then)
_SEEDS = {"flight_N10": 9000, "push_N20": 9001, "swing_left_N20": 9002, "tilt_N10": 9003,
          "flight_N5": 9004, "swing_right_N32": 9005}


def stress_workload(name):
    N, kw = STRESS_CASES[name]
    return N, make_workload(STRESS_B, N, seed=_SEEDS[name], **kw)
