// mpc_io.hpp -- the MPC step's input preparation, output post-processing and dense-output kernels
// (SURVEY.md §8(a) a12/a13, §8(f) rows 1-3).
//
// prepare_inputs_kernel: per env, the controller-side preparation the reference runs as ~40 small
//   FP32 torch ops before qp_former -- BaseMPCController.compute_knot_points / set_initial_state /
//   compute_reference_trajectory (base_controller.py:166-257), GaitGenerator.mpc_gait
//   (gait_generator.py:216-252) and the input assembly of MPCControllerCusadi.run
//   (mpc_controller_cusadi.py:54-95) -- fused into one thread per env that writes the 17 FP64
//   former inputs. FP32 arithmetic follows the torch op sequence: every torch op rounds, so products
//   and sums are evaluated with FP contraction off (no FMA).
// u0_wrench_kernel: u0 -> body-frame foot wrench, mpc_controller_cusadi.py:186-203, and optionally the
//   stance feed-forward joint torque J^T f (leg_controller.py:87-95) from the same registers.
// dense_scatter_kernel: CCS nonzeros -> dense (B, rows, cols), CusadiFunction.getDenseOutput
//   (CusadiFunction.py:49-58) as a direct scatter from an inverse index map.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srbd {

struct PrepArgs {
  // robot state estimate (float32): (B,3) x4, rotation (B,3,3) row-major, feet (B,2,3)
  const float *root_euler, *root_position, *ang_vel_w, *vel_w, *rotation_body, *foot_position;
  // command (float32): desired body velocity (B,3), angular velocity (B,3), height (B)
  const float *des_vel_b, *des_angvel_b, *des_height;
  // controller state, updated in place: world_position_desired (B,3), yaw_desired (B), first_run
  float *wpd, *yaw_des;
  uint8_t* first_run;
  // contact schedule: gait phase (B) + SSP/DSP durations (B,2) int32, or an explicit (B,N,2) table
  const float* gait_phase;
  const int32_t *ssp, *dsp;
  const float* contact_table;
  // per-env parameters (float32): dt_mpc (B), residual accelerations (B,3) x2
  const float *dt_mpc, *res_lin, *res_ang;
  float I_body[9];
  double mass, mu;
  float Q[13], R[12];
  int q_len;       // entries of the configured Q (MPCConf.Q has 13)
  float step_dt;   // float32(decimation * dt): open-loop knot advance per MPC update
  int literal;     // 1: reference GPU-caller flattening; 0: corrected layout
  double* out[17];
  int N, batch;
};

// One rounding per torch op: hipcc contracts a*b+c into an FMA by default (-ffp-contract=fast) and
// HIP's __fmul_rn/__fadd_rn are plain operations, so contraction is switched off where they live.
__device__ __forceinline__ float fm(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ float fa(float a, float b) {
#pragma clang fp contract(off)
  return a + b;
}
__device__ __forceinline__ float fa_(float a, float b) { return fa(a, b); }
// (M v)_i of a 3x3 row-major FP32 matrix as a batched matmul of one row: ((m0 v0 + m1 v1) + m2 v2)
__device__ __forceinline__ float dot3f(float m0, float m1, float m2, float v0, float v1, float v2) {
#pragma clang fp contract(off)
  return (m0 * v0 + m1 * v1) + m2 * v2;
}

// One env by the 64 lanes of one wave: the per-env scalars are wave-uniform, and the lanes write
// each output row contiguously; lane 0 alone updates the knot-point state. o[i] = env e's row of
// former input i: global memory (prepare_inputs_kernel) or the fused controller step's LDS
// (pdipm_srbd_reg.hpp), the same arithmetic either way.
__device__ inline void prepare_env(const PrepArgs& a, int e, int lane, double* const (&o)[17]) {
  const int N = a.N;
  // ---- every global load of this env first, independent of each other: one memory round trip
  // (the fused controller step runs this in front of the solve, where its latency is exposed) ----
  const float* rp = a.root_position + 3 * e;
  const float* eu = a.root_euler + 3 * e;
  const bool first = a.first_run[e] != 0;  // every lane reads it before lane 0 clears it (one stream)
  const float rp0 = rp[0], rp1 = rp[1], eu2 = eu[2];
  const float wpd0 = a.wpd[3 * e], wpd1 = a.wpd[3 * e + 1], ydes = a.yaw_des[e];
  const float* vb = a.des_vel_b + 3 * e;
  const float vb0 = vb[0], vb1 = vb[1], vb2 = vb[2];
  const float wz = a.des_angvel_b[3 * e + 2], h = a.des_height[e], dt = a.dt_mpc[e];
  float Rm[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) Rm[k] = a.rotation_body[9 * (size_t)e + k];
  const int j3 = lane % 3, g4 = lane / 3;  // lanes 0..11: x0 entry j3 of group g4
  const float* x0src = g4 == 0 ? eu : g4 == 1 ? rp : g4 == 2 ? a.ang_vel_w + 3 * e : a.vel_w + 3 * e;
  const float x0v = x0src[j3];
  const float rpj = rp[j3], flj = a.foot_position[6 * e + j3], frj = a.foot_position[6 * e + 3 + j3];
  const float rlj = a.res_lin[3 * e + j3], raj = a.res_ang[3 * e + j3];
  float phase = 0.0f;
  int s0 = 0, s1 = 0, d0 = 0, d1 = 0;
  float tl = 0.0f, tr = 0.0f;
  if (a.gait_phase) {  // uniform
    phase = a.gait_phase[e];
    s0 = a.ssp[2 * e];
    s1 = a.ssp[2 * e + 1];
    d0 = a.dsp[2 * e];
    d1 = a.dsp[2 * e + 1];
  } else if (lane < N) {
    tl = a.contact_table[(size_t)e * 2 * N + 2 * lane];
    tr = a.contact_table[(size_t)e * 2 * N + 2 * lane + 1];
  }
  // ---- compute_knot_points (base_controller.py:166-176) ----
  float w0 = first ? rp0 : wpd0, w1 = first ? rp1 : wpd1;
  float yaw = first ? eu2 : ydes;
  // compute_reference_trajectory (:213-257)
  w0 = fa(w0, fm(a.step_dt, vb0));
  w1 = fa(w1, fm(a.step_dt, vb1));
  yaw = fa(yaw, fm(a.step_dt, wz));
  const bool stationary = fabsf(vb0) < 1e-2f;
  const float vw0 = dot3f(Rm[0], Rm[1], Rm[2], vb0, vb1, vb2);
  const float vw1 = dot3f(Rm[3], Rm[4], Rm[5], vb0, vb1, vb2);
  const float px = stationary ? w0 : rp0, py = stationary ? w1 : rp1;
  if (lane == 0) {
    a.wpd[3 * e] = w0;
    a.wpd[3 * e + 1] = w1;
    a.wpd[3 * e + 2] = h;
    a.yaw_des[e] = yaw;
    a.first_run[e] = 0;
    o[4][0] = (double)dt;
    o[5][0] = a.mass;
    o[6][0] = a.mu;
  }
  // x_ref (input 3) and the linearisation points x, u = ones (mpc_controller_cusadi.py:55-57)
  double* xr = o[3];
  for (int q = lane; q < 12 * N; q += 64) {
    const int k = q / 12, j = q % 12;
    const float t = fm(dt, (float)k);
    float v;
    switch (j) {
      case 2: v = fa(yaw, fm(wz, t)); break;
      case 3: v = fa(px, fm(vw0, t)); break;
      case 4: v = fa(py, fm(vw1, t)); break;
      case 5: v = h; break;
      case 8: v = wz; break;
      case 9: v = vw0; break;
      case 10: v = vw1; break;
      default: v = 0.0f; break;
    }
    xr[q] = v;
    o[1][q] = 1.0;
    o[2][q] = 1.0;
  }
  if (lane < 12) {  // set_initial_state (:201-211) -> x0; Q, R (:70-71)
    o[0][lane] = x0v;
    // the caller hands a (B, 13) Q to an input read with stride 12, so env e sees
    // Q[(12 e + j) mod 13]; written here into a well-formed (B, 12)
    const int qi = (a.literal && a.q_len == 13) ? (int)(((long long)12 * e + lane) % 13) : lane;
    o[13][lane] = a.Q[qi];
    o[14][lane] = a.R[lane];
  } else if (lane < 21) {  // R_body (:58): row-major flattening (literal) or column-major; I_world
    const int l = lane - 12, i = l / 3, j = l % 3;
    float Ri[3], Rj[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {  // rows i and j of R, selected from registers
      Ri[k] = i == 0 ? Rm[k] : i == 1 ? Rm[3 + k] : Rm[6 + k];
      Rj[k] = j == 0 ? Rm[k] : j == 1 ? Rm[3 + k] : Rm[6 + k];
    }
    o[7][a.literal ? 3 * i + j : 3 * j + i] = j == 0 ? Ri[0] : j == 1 ? Ri[1] : Ri[2];
    // I_world = R I_body R^T as two FP32 batched matmuls (:59-61): row i of T = R I_body first
    float T[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) T[k] = dot3f(Ri[0], Ri[1], Ri[2], a.I_body[k], a.I_body[3 + k], a.I_body[6 + k]);
    o[8][3 * i + j] = dot3f(T[0], T[1], T[2], Rj[0], Rj[1], Rj[2]);
  } else if (lane < 24) {
    const int j = lane - 21;
    o[9][j] = rpj;
    o[10][j] = flj;
    o[11][j] = frj;
    o[15][j] = rlj;
    o[16][j] = raj;
  }
  // contact schedule: GaitGenerator.mpc_gait (gait_generator.py:216-252) or the given table;
  // flattened (N,2) row-major as the caller does (:65; literal) or column-major (corrected)
  double* ct = o[12];
  for (int k = lane; k < N; k += 64) {
    double cl, cr;
    if (a.gait_phase) {
      const int cyc = s0 + s1 + d0 + d1;
      if (cyc <= 0) {  // degenerate durations (torch would fault on % 0): double support
        cl = cr = 1.0;
      } else {
        const int g = (int)fm(phase, (float)cyc);  // (phase * cycle).int(): truncation
        int st = (g + k) % cyc;
        if (st < 0) st += cyc;  // torch remainder takes the divisor's sign
        const bool p1 = st < s1, p2 = st >= s1 && st < s1 + d0, p3 = st >= s1 + d0 && st < s1 + d0 + s0;
        const bool fin = !(p1 || p2 || p3);
        cl = (p1 || p2 || fin) ? 1.0 : 0.0;
        cr = (p2 || p3 || fin) ? 1.0 : 0.0;
      }
    } else {
      cl = k == lane ? tl : a.contact_table[(size_t)e * 2 * N + 2 * k];
      cr = k == lane ? tr : a.contact_table[(size_t)e * 2 * N + 2 * k + 1];
    }
    ct[a.literal ? 2 * k : k] = cl;
    ct[a.literal ? 2 * k + 1 : N + k] = cr;
  }
}

// per-env row widths of the 17 former inputs (srbd_constraints.py:77)
__host__ __device__ inline int former_in_nnz(int i, int N) {
  return (i == 1 || i == 2 || i == 3) ? 12 * N : i == 12 ? 2 * N : (i >= 4 && i <= 6) ? 1 : (i == 7 || i == 8) ? 9
       : (i == 0 || i == 13 || i == 14) ? 12 : 3;
}

#ifndef SRBD_NO_GENERAL_KERNEL  // the global kernels live in srbd_mpc.hip's unit only
// 4 envs per 256-thread block, one wave each, rows written to the global former inputs
__global__ __launch_bounds__(256) void prepare_inputs_kernel(PrepArgs a) {
  const int lane = threadIdx.x & 63;
  const int e = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (e >= a.batch) return;
  double* o[17];
#pragma unroll
  for (int i = 0; i < 17; ++i) o[i] = a.out[i] + (size_t)e * former_in_nnz(i, a.N);
  prepare_env(a, e, lane, o);
}

#endif

// The foot wrench of one env from its first-stage input u0 (12 doubles, FP32 after the cast the
// caller applies): lane j < 12 computes w[j] = -(R^T v)_i of block j / 3 (mpc_controller_cusadi.py:
// 186-203, u = [lf, rf, lm, rm] -> w = [lf, lm | rf, rm], x-moments zeroed); one value per lane.
__device__ __forceinline__ float wrench_entry(const double* u0, const float* Rm, int j) {
  const int src[4] = {0, 6, 3, 9};
  const int b = j / 3, i = j % 3, s = src[b];
  float v[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) v[k] = (s + k == 6 || s + k == 9) ? 0.0f : (float)u0[s + k];
  return -dot3f(Rm[i], Rm[3 + i], Rm[6 + i], v[0], v[1], v[2]);
}

#ifndef SRBD_NO_GENERAL_KERNEL
// u0 -> body-frame foot wrench (float32, (B, 2, 6)): mpc_controller_cusadi.py:186-203
__global__ __launch_bounds__(256) void u0_wrench_kernel(int N, int batch, const double* __restrict__ x,
                                                        const float* __restrict__ rotation_body,
                                                        float* __restrict__ wrench, int ndof,
                                                        const float* __restrict__ J,
                                                        const float* __restrict__ contact,
                                                        float* __restrict__ tau) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= batch) return;
  const double* u0 = x + (size_t)e * 24 * N + 12 * N;
  float u[12];
  for (int j = 0; j < 12; ++j) u[j] = (float)u0[j];
  u[6] = 0.0f;  // left_grm[:, 0] = 0
  u[9] = 0.0f;  // right_grm[:, 0] = 0
  const float* Rm = rotation_body + 9 * e;
  float w[12];
  // R^T v, then negate; blocks [lf, lm | rf, rm] with u = [lf(0..2), rf(3..5), lm(6..8), rm(9..11)]
  const int src[4] = {0, 6, 3, 9};
  for (int b = 0; b < 4; ++b) {
    const float* v = u + src[b];
    for (int i = 0; i < 3; ++i) w[3 * b + i] = -dot3f(Rm[i], Rm[3 + i], Rm[6 + i], v[0], v[1], v[2]);
  }
  for (int j = 0; j < 12; ++j) wrench[(size_t)e * 12 + j] = w[j];
  if (!tau) return;
  // stance feed-forward torque, LegController.update_ff_torque (leg_controller.py:87-95):
  // tau_l = contact_l ? J_l^T f_l : 0 with J (B,2,6,ndof) and f_l = wrench row l; the 6-term
  // reduction runs in index order, one rounding per op
  for (int l = 0; l < 2; ++l) {
    const bool on = contact[(size_t)e * 2 + l] != 0.0f;
    const float* Jl = J + ((size_t)e * 2 + l) * 6 * ndof;
    for (int k = 0; k < ndof; ++k) {
      float t = 0.0f;
      if (on) {
        t = fm(Jl[k], w[6 * l]);
        for (int j = 1; j < 6; ++j) t = fa(t, fm(Jl[j * ndof + k], w[6 * l + j]));
      }
      tau[((size_t)e * 2 + l) * ndof + k] = t;
    }
  }
}

// dense (B, rc) from CCS nonzeros (B, nnz) through inv[rc] (nonzero index or -1); each thread
// writes two consecutive entries with one 16-byte store when rc is even (every env's row is then
// 16-byte aligned), one 8-byte store otherwise
__global__ __launch_bounds__(256) void dense_scatter_kernel(int rc, int nnz, int batch, const int32_t* __restrict__ inv,
                                                            const double* __restrict__ vals,
                                                            double* __restrict__ dense) {
  const int e = blockIdx.y;
  if (e >= batch) return;
  const double* v = vals + (size_t)e * nnz;
  double* out = dense + (size_t)e * rc;
  if ((rc & 1) == 0) {
    const int i0 = 2 * (blockIdx.x * blockDim.x + threadIdx.x);
    if (i0 >= rc) return;
    const int2 k = *reinterpret_cast<const int2*>(inv + i0);
    double2 r;
    r.x = k.x >= 0 ? v[k.x] : 0.0;
    r.y = k.y >= 0 ? v[k.y] : 0.0;
    *reinterpret_cast<double2*>(out + i0) = r;
  } else {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < rc; i += gridDim.x * blockDim.x) {
      const int k = inv[i];
      out[i] = k >= 0 ? v[k] : 0.0;
    }
  }
}

#endif

}  // namespace srbd
