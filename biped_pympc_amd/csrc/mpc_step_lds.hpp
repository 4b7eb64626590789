// mpc_step_lds.hpp -- the one-launch MPC step at ANY horizon (1 <= N <= 32): input preparation
// (controller step) or the 17 former inputs, qp_former's model, the cold-started PDIPM of the
// LDS-resident stage-invariant kernel (pdipm_srbd.hpp FastCtx) and the u0 -> wrench (+ stance
// torque) epilogue, in ONE kernel. The register kernels (pdipm_srbd_reg.hpp mpc_step_reg_kernel) do
// this at N = 10 and 20; every other horizon runs here instead of three launches (srbd_prepare_inputs
// -> qp_former -> solver -> srbd_u0_wrench_torque). The reference regenerates and recompiles its
// CusADi kernels per horizon (srbd_constraints.py:10, README.md:80-84).
//
// Bit-identical to qp_former -> pdipm_srbd_kernel (-> u0_wrench_kernel): the stage blocks come from
// the former's own device code (former_model, former_f / former_b / former_d / former_g) and the
// solver is the same FastCtx, with f, h, b and the refinement's saved dx / dy in LDS instead of
// memory. The QP never reaches HBM unless the caller asks for f, b, d (fa.vec).
#pragma once
#include "pdipm_srbd_reg.hpp"  // FusedArgs, prepare_env, wrench_entry

namespace srbd {

__host__ __device__ inline size_t step_lds_bytes(int N) { return sizeof(double) * (size_t)FastLayout(N, true).total; }

template <int NT>
__global__ __launch_bounds__(64) void mpc_step_lds_kernel(FusedArgs fa) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int env = xcd_item(blockIdx.x, gridDim.x);
  if (env >= fa.batch) return;
  const int N = NT > 0 ? NT : fa.N, lane = threadIdx.x;
  const int nz = 24 * N, m = 16 * N, p = 14 * N, nx = 12 * N;
  const FastLayout Lo(N, true);
  FastCtx<NT> C;
  C.N_ = N;
  C.lane = lane;
  C.bind(smem, Lo);
  // ---- this env's 17 former inputs in FI: prepared here (controller step) or staged from memory ----
  const double* P[17];
  double* o[17];
  {
    int off = 0;
#pragma unroll
    for (int i = 0; i < 17; ++i) {
      o[i] = smem + Lo.FI + off;
      P[i] = o[i];
      off += former_in_nnz(i, N);
    }
  }
  if (fa.ctrl) {
    prepare_env(fa.prep, env, lane, o);
    __syncthreads();
    if (fa.prep.out[0]) {  // the caller also wants the prepared inputs in memory
#pragma unroll
      for (int i = 0; i < 17; ++i) {
        const int w = former_in_nnz(i, N);
        double* g = fa.prep.out[i] + (size_t)env * w;
        for (int e = lane; e < w; e += 64) g[e] = o[i][e];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 17; ++i) {
      const int w = former_in_nnz(i, N);
      const double* g = fa.in[i] + (size_t)env * w;
      for (int e = lane; e < w; e += 64) o[i][e] = g[e];
    }
    __syncthreads();
  }
  // ---- the discrete model (qp_former's device code) and the stage blocks ----
  FormerLds& F = *reinterpret_cast<FormerLds*>(smem + Lo.RX);  // RX .. SC are dead until the iterations
  former_model(F, P, lane);
  const double mu = P[6][0];
  for (int e = lane; e < 144; e += 64) {
    const int r = e / 12, j = e % 12;
    const int om = c_tab.Mi[r][j], on = c_tab.Ni[r][j];
    C.Md[e] = (N >= 2 && om >= 0) ? F.XB[om] : 0.0;
    C.Nd[e] = on >= 0 ? F.UB[on] : 0.0;
  }
  for (int e = lane; e < 192; e += 64) C.Gd[e] = 0.0;
  if (lane < 12) {
    C.Pd[lane] = F.XB[c_tab.cpx[lane]];
    C.Hu[lane] = P[14][lane];       // H = diag(Q.., R..): u part R
    C.Hu[12 + lane] = P[13][lane];  // x part Q
  }
  const double e6 = F.UB[c_tab.e6], e9 = F.UB[c_tab.e9];
  double *FV = smem + Lo.FV, *HV = smem + Lo.HV, *BV = smem + Lo.BV;
  for (int e = lane; e < nz; e += 64) FV[e] = former_f(e, N, P[13], P[14], P[1], P[2], P[3]);
  for (int e = lane; e < m; e += 64) HV[e] = former_d(e, N, P[2], P[12], mu);
  for (int e = lane; e < p; e += 64) BV[e] = former_b(e, N, F);
  __syncthreads();
  if (lane < 28) C.Gd[c_tab.grow[lane] * 12 + c_tab.gcol[lane]] = former_g(lane, mu);
  if (fa.vec[0])
    for (int e = lane; e < nz; e += 64) fa.vec[0][(size_t)env * nz + e] = FV[e];
  if (fa.vec[1])
    for (int e = lane; e < p; e += 64) fa.vec[1][(size_t)env * p + e] = BV[e];
  if (fa.vec[2])
    for (int e = lane; e < m; e += 64) fa.vec[2][(size_t)env * m + e] = HV[e];
  C.fg = FV;
  C.hg = HV;
  C.bg = BV;
  C.xsg = smem + Lo.XS;
  C.ysg = smem + Lo.YS;
  C.constants(e6, e9);
  // ---- cold start (mpc_controller_cusadi.py:138-141) and the Newton loop ----
  for (int e = lane; e < nz; e += 64) C.X[e] = 0.0;
  for (int e = lane; e < m; e += 64) {
    C.S[e] = fmax(HV[e] - 0.0, 1.0);
    C.Z[e] = 1.0;
  }
  for (int e = lane; e < p; e += 64) C.Y[e] = fa.y0;
  __syncthreads();
  double res[4] = {0.0, 0.0, 0.0, 0.0};
  bool floor_hit = false;
  C.newton(fa.n_iter, res, floor_hit);
  if (fa.status) {
    const int st = C.status(res[3], floor_hit);
    if (lane == 0) fa.status[env] = st;
  }
  // ---- outputs (each optional) ----
  if (double* xo = fa.out[0])
    for (int e = lane; e < nz; e += 64) xo[(size_t)env * nz + e] = C.X[e];
  if (double* so = fa.out[1])
    for (int e = lane; e < m; e += 64) so[(size_t)env * m + e] = C.S[e];
  if (double* zo = fa.out[2])
    for (int e = lane; e < m; e += 64) zo[(size_t)env * m + e] = C.Z[e];
  if (double* yo = fa.out[3])
    for (int e = lane; e < p; e += 64) yo[(size_t)env * p + e] = C.Y[e];
  if (lane == 0) {
    if (double* ro = fa.out[4]) {
#pragma unroll
      for (int k = 0; k < 4; ++k) ro[(size_t)env * 4 + k] = res[k];
    }
    if (double* mo = fa.out[5]) mo[env] = res[3];
  }
  if (fa.wrench) {  // u0 -> foot wrench (+ stance torque): srbd_u0_wrench_torque's arithmetic
    const float* Rm = fa.prep.rotation_body + 9 * (size_t)env;
    float* wl = reinterpret_cast<float*>(C.TV);  // TV is dead after the last update
    if (lane < 12) {
      const float w = wrench_entry(C.X + nx, Rm, lane);
      fa.wrench[(size_t)env * 12 + lane] = w;
      wl[lane] = w;
    }
    if (fa.tau) {
      __syncthreads();
      const int nd = fa.ndof;
      for (int q = lane; q < 2 * nd; q += 64) {
        const int l = q / nd, k = q - l * nd;
        const float* Jl = fa.jac + ((size_t)env * 2 + l) * 6 * nd;
        float t = 0.0f;
        if (fa.contact[(size_t)env * 2 + l] != 0.0f) {
          t = fm(Jl[k], wl[6 * l]);
          for (int j = 1; j < 6; ++j) t = fa_(t, fm(Jl[j * nd + k], wl[6 * l + j]));
        }
        fa.tau[((size_t)env * 2 + l) * nd + k] = t;
      }
    }
  }
}

}  // namespace srbd
