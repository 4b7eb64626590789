/*
 * srbd_mpc.h -- C-ABI of the MI355X-native SRBD-MPC QP engine (libsrbd_mpc.so + thin drop-ins).
 *
 * Drop-in boundary for the reference's CusADi hot path (rl-augmented-mpc/Biped-PyMPC):
 *   - `evaluate` below is the exact symbol each CusADi function library exports
 *     (reference biped_pympc/cusadi/src/generateCUDACode.py:157-183) and that
 *     CusadiFunction binds through ctypes (biped_pympc/cusadi/src/CusadiFunction.py:28-47).
 *     Two thin libraries export it: libqp_former.so (CasADi Function 'qp_former',
 *     srbd_constraints.py:75-79) and libsparse_pdipm_multiple_iterations.so ('sparse_pdipm_multiple_iterations',
 *     sparse_pdipm_solver.py:532-534), built for the deployed configuration N = 10, 5 iterations
 *     (mpc_controller_cusadi.py:28; generate_solver_function.py:106). Other horizons/iteration counts
 *     get libqp_former_N<N>.so / libsparse_pdipm_multiple_iterations_N<N>_K<K>.so.
 *   - the srbd_* entry points are the extended API (runtime horizon and iteration count, caller's
 *     HIP stream, fused former+solve), all plain pointers and sizes.
 *
 * Memory: every double* is DEVICE memory, batched row-major (batch, nnz) per tensor, exactly the
 * CusADi layout (input i of env e at inputs[i] + e*nnz_in[i]). The library allocates nothing on
 * the device; it never calls exit(): failures return an error code and set srbd_last_error().
 */
#ifndef SRBD_MPC_H_
#define SRBD_MPC_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRBD_ABI_VERSION 1
#define SRBD_MAX_HORIZON 32

/* ---- CusADi ABI (thin per-function libraries) ---------------------------------------------
 * inputs/outputs: DEVICE pointer to a DEVICE array of n_in / n_out DEVICE pointers
 * (CusadiFunction.py:84-92). work: ignored (CusADi's (batch, sz_w) scratch; may be NULL).
 * Blocking, legacy default stream. Returns kernel time in SECONDS (generateCUDACode.py:176-182),
 * or a negative value on error (the reference's gpuErrchk calls exit(); this never does). */
float evaluate(const double* inputs[], double* work, double* outputs[], const int batch_size);

/* ---- Extended API (libsrbd_mpc.so) ------------------------------------------------------------ */
int srbd_abi_version(void);
const char* srbd_last_error(void);
/* Build provenance: 16 hex digits of sha256 over the library's sources and compile flags
 * (biped_pympc_amd/build.py source_hash); smoke() and bench.py print it. */
const char* srbd_build_id(void);

/* CusADi-ABI implementations with explicit configuration (what the thin libraries call). */
float srbd_evaluate_qp_former(int horizon, const double* inputs[], double* work, double* outputs[],
                              int batch);
float srbd_evaluate_pdipm(int horizon, int n_iter, const double* inputs[], double* work,
                          double* outputs[], int batch);

/* qp_former: 17 inputs (x0, x, u, x_ref, dt, m, mu, R_body, I_world, body_pos, left_foot_pos,
 * right_foot_pos, contact_table, Q, R, residual_lin_accel, residual_ang_accel;
 * srbd_constraints.py:77) -> 6 outputs (nonzeros of H, f, A, b, G, d in CCS order).
 * `inputs`/`outputs` are HOST arrays of device pointers. Asynchronous on `stream` (hipStream_t,
 * NULL = default stream). Returns 0 or a hipError_t code. */
int srbd_qp_former(int horizon, int batch, const double* const* inputs, double* const* outputs,
                   void* stream);

/* sparse PDIPM: 10 inputs (Q_val, G_val, A_val, f, h, b, x, s, z, y; sparse_pdipm_solver.py:533)
 * -> 6 outputs (x, s, z, y, residuals[4] = [|rx|, |rs|, |re|, mu_new], mu_new), n_iter >= 1
 * Newton iterations at run time. Host array of device pointers; asynchronous on `stream`. */
int srbd_pdipm(int horizon, int n_iter, int batch, const double* const* inputs,
               double* const* outputs, void* stream);

/* Same, but the iterate is initialised on device as the GPU caller does
 * (mpc_controller_cusadi.py:138-141): x = 0, s = max(h, 1), z = 1, y = y0. Inputs 6..9 unused
 * (may be NULL). */
int srbd_pdipm_cold(int horizon, int n_iter, int batch, double y0, const double* const* inputs,
                    double* const* outputs, void* stream);

/* The reference's `_ccs` solver entry (sparse_pdipm_solver_ccs, sparse_pdipm_solver.py:4-35, and
 * initialize_pdipm_variables :537-558): the iterate starts from an arbitrary primal guess,
 * x = x_init (input 6), s = max(h - G x_init, 1), z = 1, y = 0; inputs 7..9 unused (may be NULL).
 * The reference Function returns x only; here all 6 outputs as srbd_pdipm. */
int srbd_pdipm_ccs(int horizon, int n_iter, int batch, const double* const* inputs, double* const* outputs,
                   void* stream);

/* Per-problem status word (failure detection; the reference has no such output, only its
 * clamps, sparse_pdipm_solver.py:466-467,501-515): int32 per env, OR of
 *   SRBD_STATUS_NONFINITE  a NaN / Inf in the returned x, s, z, y or mu
 *   SRBD_STATUS_STEP_FLOOR a combined-direction step length (primal or dual) at its 1e-12 floor in the
 *                          last iteration (the iterate is stalled at the boundary)
 *   SRBD_STATUS_FALLBACK   the QP was not stage-invariant and a stage-invariant kernel (solver path
 *                          "auto" or "lds") solved it by its in-launch general fallback; set only there:
 *                          under the "general" path (srbd_set_solver_path(1)) every QP takes the general
 *                          kernel and this bit stays clear
 * Written by the *_ex entry points when status != NULL (device memory, batch ints). */
#define SRBD_STATUS_NONFINITE 1
#define SRBD_STATUS_STEP_FLOOR 2
#define SRBD_STATUS_FALLBACK 4

/* srbd_pdipm (init_mode 0), srbd_pdipm_cold (1, y = y0) or srbd_pdipm_ccs (2) with the status word. */
int srbd_pdipm_ex(int horizon, int n_iter, int batch, int init_mode, double y0, const double* const* inputs,
                  double* const* outputs, int* status, void* stream);

/* Whole MPC QP step: qp_former -> cold-start PDIPM (n_iter iterations), one stream, no host sync.
 * `qp_workspace` is caller-owned device memory of srbd_mpc_workspace_doubles(horizon, batch)
 * doubles that receives H, f, A, b, G, d (CCS, batched). outputs as srbd_pdipm. */
size_t srbd_mpc_workspace_doubles(int horizon, int batch);
int srbd_mpc_solve(int horizon, int n_iter, int batch, double y0, const double* const* former_inputs,
                   double* qp_workspace, double* const* outputs, void* stream);

/* srbd_mpc_solve in ONE kernel at every horizon (the register kernels at N = 2..32, the
 * LDS-resident step kernel otherwise; a non-auto solver path runs srbd_mpc_solve and needs
 * qp_workspace): the QP is formed in the solver from the former inputs and never written, except
 * f, b, d into their qp_workspace slots when qp_workspace != NULL (NULL: no QP data leaves the
 * kernel). Same outputs as srbd_mpc_solve, bit for bit; any outputs[k] may be NULL (that output is
 * not written). */
int srbd_mpc_solve_fused(int horizon, int n_iter, int batch, double y0, const double* const* former_inputs,
                         double* qp_workspace, double* const* outputs, void* stream);
/* srbd_mpc_solve_fused with the status word (status may be NULL). */
int srbd_mpc_solve_fused_ex(int horizon, int n_iter, int batch, double y0, const double* const* former_inputs,
                            double* qp_workspace, double* const* outputs, int* status, void* stream);

/* LDS bytes one solver workgroup (one QP) uses at this horizon (0 if unsupported). */
size_t srbd_solver_lds_bytes(int horizon);

/* Solver kernel selection: 0 = auto (default): a stage-invariant kernel for stage-invariant QPs
 * (every QP qp_former emits; register-resident at N = 2..32, LDS-resident otherwise), the general
 * kernel for any other QP in the batch; 1 = general kernel only; 2 = LDS-resident stage-invariant
 * kernel at every horizon (plus the general fallback).
 * Results agree to round-off (tests/test_gpu_parity.py). Per device: applies to calls made while
 * the current HIP device is the one current here.
 *
 * Devices: every entry point works on the HIP device current at the call (one process per GPU is
 * the deployment model; a process that switches devices is supported too). What the
 * library keeps between calls -- configured kernel LDS limits, the blocking calls' events, the
 * solver path -- is kept per device (csrc/device_state.hpp). */
int srbd_set_solver_path(int path);
/* The solver path in effect for the current HIP device (0 if never set). srbd_mpc_solve_fused under a
 * non-auto path runs srbd_mpc_solve and so needs qp_workspace; srbd_mpc_step ignores the path and
 * always runs its one-launch step kernel (its QPs are stage-invariant by construction): the
 * register-resident kernel at N = 2..32, the LDS-resident step kernel at N = 1. */
int srbd_get_solver_path(void);

/* Affine-direction refinement of the register-resident kernels (the default solvers at N = 2..32), per
 * device like the solver path. Every Newton iteration refines the combined direction once against the
 * full KKT; the affine (predictor) direction, whose ds / dz set sigma and the corrector, is refined
 * 0 = (default) at the iterate a solve starts from (every dual z at its initial 1: the cold start's Newton
 *     step is the largest) and in iterations with an ill-conditioned iterate (some row with z / s >= 1e4
 *     or an s at its 1e-8 clamp) -- where an unrefined predictor lets the trajectory drift from the
 *     reference's; about the time at N = 10 of round 5's mode 0 (predictor at z / s >= 1e3 only);
 * 1 = in every iteration (as the LDS-resident and general kernels always do), ~15 % more time at N = 10.
 * scripts/parity_fuzz.py + scripts/parity_floor.py, every env above the tolerance floor-checked, 6657 cases
 * of each sequence: mode 0 fails a few register-kernel warm starts, mode 1 none (DESIGN.md 3.3 has the
 * counts), round 5's mode 0 23 and 26 -- a case fails when an env sits more than 4x its FP64 floor (the
 * larger distance of the AMD-ordered LDL^T and of dense LU from the checker) beyond the K tolerance; no env
 * of either mode is over 1e-4 relative in x or u0 beyond that (profiles/r06/). Returns 0, or
 * an error for another mode. */
int srbd_set_refinement(int mode);
/* The refinement mode in effect for the current HIP device (0 if never set; 2 after
 * srbd_set_refinement_policy). */
int srbd_get_refinement(void);

/* Diagnostics (A/B campaigns, scripts/parity_fuzz.py): an explicit refinement policy for the register
 * kernels on the current device, in place of the mode. flags: SRBD_REFINE_AFFINE_ALL (the affine
 * direction in every iteration), SRBD_REFINE_AFFINE_AT_INIT (at an iterate whose duals z are all 1: the
 * initial iterate of the GPU caller's and of the _ccs init), SRBD_REFINE_AFFINE_FIRST(k) /
 * SRBD_REFINE_AFFINE_LAST(k) (in the first / last k iterations of a call -- position-based: chained calls
 * then no longer equal one long call); w: the affine vote's W = z / s threshold (w <= 0: no W vote; an s
 * at its clamp always votes). Mode 0 is SRBD_REFINE_AFFINE_AT_INIT with w = 1e4, mode 1
 * SRBD_REFINE_AFFINE_ALL. The
 * combined direction is refined in every iteration whatever the policy. srbd_set_refinement(mode)
 * returns to a mode. Returns 0, or an error for unknown bits or a NaN threshold. */
#define SRBD_REFINE_AFFINE_ALL 1
#define SRBD_REFINE_AFFINE_AT_INIT 2
#define SRBD_REFINE_AFFINE_FIRST(k) (((k) & 255) << 8)
#define SRBD_REFINE_AFFINE_LAST(k) (((k) & 255) << 16)
int srbd_set_refinement_policy(int flags, double w);

/* Allocates what the solver entry points keep per device -- the general-fallback scratch pool of the
 * stage-invariant kernels (one slot per resident workgroup -- 2048 on an MI355X of
 * srbd_scratch_slot_bytes() = 162,000 B each: 332 MB of HBM per process and device, lock words
 * included) -- on the current HIP
 * device, synchronising it. Optional: the first srbd_pdipm* / srbd_mpc_solve* / evaluate call on a
 * device does the same, but that first call must then not be made inside a stream capture (it returns
 * an error there): call this, or make one ordinary call, before capturing a graph. Returns 0 or an
 * error code. (The pool's lock words are released by the workgroups that take them; a kernel that
 * faults leaves the HIP context unusable anyway.) */
int srbd_prepare_device(void);

/* Frees the current device's scratch pool after synchronising the device (the next solver call, or
 * srbd_prepare_device, allocates it again). Graphs captured before still hold the old pool's address:
 * do not replay them afterwards. Returns 0 or an error code. */
int srbd_release_device(void);

/* Caps the current device's pool at `slots` (>= 1; 0 = the default, one per resident workgroup) for
 * processes that share a GPU; the environment variable SRBD_SCRATCH_SLOTS does the same when no cap
 * is set. Any count >= 1 is correct: a QP that is not stage-invariant and finds every slot taken
 * waits for one. A pool of another size is released (device synchronised) and re-allocated on the
 * next call. */
int srbd_set_scratch_slots(int slots);

/* Bytes / slots of the current device's pool (0 before it is allocated), and the bytes of one slot
 * (host-only: no device needed). */
size_t srbd_scratch_pool_bytes(void);
int srbd_scratch_pool_slots(void);
size_t srbd_scratch_slot_bytes(void);

/* Host-only introspection: rebuild the CCS pattern of H (which = 0), A (1) or G (2) from the very
 * offset maps the kernels use to address A_val/G_val. colptr has 24*horizon+1 entries, rowind nnz.
 * Returns nnz, or a negative value if the kernel's offsets are not a bijection onto a sorted CCS. */
int srbd_pattern_ccs(int horizon, int which, int* colptr, int* rowind);

/* ---- MPC step around the QP ------------------------ */

/* Everything BaseMPCController / MPCControllerCusadi assemble on the host before qp_former, as
 * device arrays (float32 unless noted, batch-major). Field groups mirror the reference data
 * classes: StateEStimatorData and DesiredStateData (core/data/robot_data.py:9-60), the controller's
 * own knot-point state (base_controller.py:48,71-72), GaitGenerator (gait_generator.py:4-76) and
 * MPCConf / the robot model (configuration.py:23-57, core/robot/hector.py:33-38). */
typedef struct srbd_mpc_prep {
  const float* root_euler;                 /* (B,3) */
  const float* root_position;              /* (B,3) */
  const float* root_angular_velocity_w;    /* (B,3) */
  const float* root_velocity_w;            /* (B,3) */
  const float* rotation_body;              /* (B,3,3) row-major */
  const float* foot_position;              /* (B,2,3) world frame, [left, right] */
  const float* desired_velocity_b;         /* (B,3) */
  const float* desired_angular_velocity_b; /* (B,3) */
  const float* desired_height;             /* (B) */
  float* world_position_desired;           /* (B,3) read + updated */
  float* yaw_desired;                      /* (B)   read + updated */
  unsigned char* first_run;                /* (B)   bool, read + cleared */
  const float* gait_phase;                 /* (B) or NULL: then contact_table is used */
  const int* ssp_durations;                /* (B,2) int32 [left, right] */
  const int* dsp_durations;                /* (B,2) int32 */
  const float* contact_table;              /* (B,N,2), used when gait_phase == NULL */
  const float* dt_mpc;                     /* (B) */
  const float* residual_lin_accel;         /* (B,3) */
  const float* residual_ang_accel;         /* (B,3) */
  float I_body[9];                         /* host constants: body inertia (row-major) */
  double mass, mu;
  float Q[13];                             /* MPCConf.Q (13 entries in the reference config) */
  int q_len;                               /* 12 or 13 */
  float R[12];
  float step_dt;                           /* float32(decimation * dt) */
  int literal_layout;                      /* 1 = the reference GPU caller's flattening of R_body,
                                              contact_table and Q;
                                              0 = corrected layout */
} srbd_mpc_prep;

/* Replaces compute_knot_points + set_initial_state + compute_reference_trajectory
 * (base_controller.py:166-257), GaitGenerator.mpc_gait (gait_generator.py:216-252) and the input
 * assembly of MPCControllerCusadi.run (mpc_controller_cusadi.py:54-95): writes the 17 qp_former
 * inputs (FP64, (B, nnz_in[i]), Q well-formed 12 wide) and updates the knot-point state. */
int srbd_prepare_inputs(int horizon, int batch, const srbd_mpc_prep* prep, double* const* former_inputs,
                        void* stream);

/* The whole controller step in ONE kernel launch (any horizon 1..32): srbd_prepare_inputs' arithmetic
 * computes this env's 17 former inputs into on-chip memory (and advances the knot-point state in
 * prep), the fused former + cold PDIPM (n_iter iterations, y = y0) solves, and
 * srbd_u0_wrench_torque's arithmetic writes foot_wrench (B,2,6) float32 -- and tau (B,2,ndof) when
 * tau != NULL, from contact_jacobian (B,2,6,ndof) / contact_bool (B,2). former_inputs (host array
 * of 17 device pointers as srbd_prepare_inputs) may be NULL: the prepared inputs then never leave
 * the chip. outputs (host array of 6 device pointers as srbd_pdipm) may be NULL, and each entry
 * may be NULL: the step then writes only the wrench (48 B/env). Bit-identical to srbd_prepare_inputs -> srbd_mpc_solve_fused ->
 * srbd_u0_wrench_torque. Replaces MPCControllerCusadi.run (mpc_controller_cusadi.py:43-205) with
 * BaseMPCController's preparation (base_controller.py:166-257) and LegController.update_ff_torque
 * (leg_controller.py:87-95). */
int srbd_mpc_step(int horizon, int n_iter, int batch, double y0, const srbd_mpc_prep* prep,
                  double* const* former_inputs, double* const* outputs, float* foot_wrench, int ndof,
                  const float* contact_jacobian, const float* contact_bool, float* tau, void* stream);
/* srbd_mpc_step with the status word (status may be NULL). */
int srbd_mpc_step_ex(int horizon, int n_iter, int batch, double y0, const srbd_mpc_prep* prep,
                     double* const* former_inputs, double* const* outputs, float* foot_wrench, int ndof,
                     const float* contact_jacobian, const float* contact_bool, float* tau, int* status,
                     void* stream);

/* u0 = x[:, 12N:12N+12] -> foot wrench (B,2,6) float32 in the body frame, x-moments zeroed and
 * negated as mpc_controller_cusadi.py:186-203. rotation_body (B,3,3) float32 row-major. */
int srbd_u0_wrench(int horizon, int batch, const double* x, const float* rotation_body, float* foot_wrench,
                   void* stream);

/* srbd_u0_wrench plus the stance feed-forward joint torque of LegController.update_ff_torque
 * (leg_controller.py:87-95; fed by BipedController._run_stance_leg_controller,
 * biped_controller.py:144-146): tau (B,2,ndof) float32 = contact_bool[b,l] != 0 ? J[b,l]^T wrench[b,l]
 * : 0, with contact_jacobian (B,2,6,ndof) and contact_bool (B,2) float32. tau == NULL skips it. */
int srbd_u0_wrench_torque(int horizon, int batch, const double* x, const float* rotation_body, float* foot_wrench,
                          int ndof, const float* contact_jacobian, const float* contact_bool, float* tau,
                          void* stream);

/* CusadiFunction.getDenseOutput (CusadiFunction.py:49-58) as one scatter: dense (B, rc) row-major
 * from nonzeros (B, nnz) through inverse_index[rc] (nonzero index of each dense entry, or -1). */
int srbd_dense_scatter(int batch, int nnz, int rc, const int* inverse_index, const double* values,
                       double* dense, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SRBD_MPC_H_ */
