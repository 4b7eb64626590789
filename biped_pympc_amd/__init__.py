"""biped_pympc_amd -- MI355X-native batched SRBD-MPC QP engine (qp_former + sparse PDIPM).

Drop-in for the hot path of rl-augmented-mpc/Biped-PyMPC: the CusADi-generated ``qp_former`` and
``sparse_pdipm_multiple_iterations`` kernels (reference ``biped_pympc/convex_mpc/
mpc_controller_cusadi.py:23-36,99,156``) are replaced by hand-written HIP kernels for gfx950 behind
a C-ABI (``include/srbd_mpc.h``), reached from Python through ``biped_pympc_amd.cusadi``.
"""
__version__ = "0.1.0"
