// pdipm_srbd.hpp -- fast PDIPM kernel for stage-invariant SRBD QPs (the ones qp_former emits).
//
// Same maths, inputs and outputs as pdipm_kernel (pdipm.hpp; reference
// biped_pympc/casadi/sparse_pdipm_solver.py:357-534). Every QP produced by qp_former has
// IDENTICAL A/G/H values in every horizon stage: the reference builds all stages from one R_body,
// one inertia and one pair of feet (srbd_constraints.py:120-126, base_controller.py:187-199), so
// -A_d, -B_d, the x-moment rows, the friction/line-contact rows and diag(Q)/diag(R) repeat. This
// kernel verifies that bitwise per QP and then keeps ONE dense copy of the stage matrices in LDS:
//   M = x_i-columns of stage i (12x12, i >= 1), N = u_i-columns (12x12), P (12), e6/e9, G (16x12),
//   H_x, H_u (12 each)
// and precomputes what does not change across stages or Newton iterations:
//   C = S_{i,i-1} = M diag(P / phi_x)          (the dual coupling block)
//   K0, K1 = constant part of S_ii for i = 0 / i >= 1 (P^2/phi_x + delta + M phi_x^-1 M^T +
//            the four decoupled u columns)
// so each iteration only rebuilds the two 4x4 foot blocks of Phi_u per stage. All inner loops have
// compile-time trip counts over dense 12-wide rows (no pattern tables, no branches).
// A QP that is not stage-invariant is left to pdipm_kernel: this kernel writes kFallbackMu into its
// mu output and pdipm_kernel (only_flagged = 1) solves exactly those.
#pragma once
#include "pdipm.hpp"

namespace srbd {


struct FastLayout {
  int Md, Nd, Cd, Gd, K0, K1, Pd, IX, Hu, SG, PH, DV, X, S, Z, Y, RX, RS, RE, WD, DI, VV, R1T, TV, QV, WV,
      DS, DZ, DY, SC, total;
  __host__ __device__ FastLayout(int N) {
    const int nz = 24 * N, m = 16 * N, p = 14 * N, nd = 12 * N;
    int o = 0;
    auto take = [&](int n) { int r = o; o += (n + 1) & ~1; return r; };
    Md = take(144); Nd = take(144); Cd = take(144); Gd = take(192);
    K0 = take(78); K1 = take(78); Pd = take(12); IX = take(12); Hu = take(24); SG = take(16);
    PH = take(20 * N); DV = take(78 * N);
    X = take(nz); S = take(m); Z = take(m); Y = take(p);
    RX = take(nz); RS = take(m); RE = take(p);
    WD = take(m); DI = take(m); VV = take(m);
    R1T = take(nz); TV = take(nz); QV = take(nd); WV = take(nd);
    DS = take(m); DZ = take(m); DY = take(p);
    SC = take(160);
    total = o;
  }
};

// packed-lower index -> (row, col), computed without loops
__device__ inline void tri_rc(int e, int& r, int& c) {
  r = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
  if ((r + 1) * (r + 2) / 2 <= e) ++r;
  if (r * (r + 1) / 2 > e) --r;
  c = e - r * (r + 1) / 2;
}

struct FastCtx {
  int N, nz, m, p, lane;
  double *Md, *Nd, *Cd, *Gd, *K0, *K1, *Pd, *IX, *Hu, *SG, *PH, *DV, *X, *S, *Z, *Y, *RX, *RS, *RE, *WD,
      *DI, *VV, *R1T, *TV, *QV, *WV, *DS, *DZ, *DY, *SC;
  const double *fg, *hg, *bg;
  // Hu: [H_u (12) | H_x (12)] ; SG: [gamma6, psi8, gamma9, psi11, phi6, phi9, e6, e9]

  __device__ double dotrow12(const double* row, const double* v) const {  // sum_j row[j] v[j]
    double a = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) a += row[j] * v[j];
    return a;
  }
  __device__ double dotcol12(const double* mat, int col, const double* v) const {  // sum_r mat[r][col] v[r]
    double a = 0.0;
#pragma unroll
    for (int r = 0; r < 12; ++r) a += mat[r * 12 + col] * v[r];
    return a;
  }

  // --------------------------------------------------------------------- residuals ----
  __device__ double residuals() {
    for (int c = lane; c < nz; c += 64) {
      double v;
      if (c < 12 * N) {
        const int k = c / 12 + 1, j = c % 12;
        v = Hu[12 + j] * X[c] + fg[c];  // Hu[12..23] holds H_x
        double ay = Pd[j] * Y[12 * (k - 1) + j];
        if (k < N) ay += dotcol12(Md, j, Y + 12 * k);
        v = v + ay;
      } else {
        const int i = (c - 12 * N) / 12, j = (c - 12 * N) % 12;
        v = Hu[j] * X[c] + fg[c];
        double gz = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) gz += Gd[k * 12 + j] * Z[16 * i + k];
        double ay = dotcol12(Nd, j, Y + 12 * i);
        if (j == 6) ay += SG[6] * Y[12 * N + 2 * i];
        if (j == 9) ay += SG[7] * Y[12 * N + 2 * i + 1];
        v = (v + gz) + ay;
      }
      RX[c] = v;
    }
    for (int e = lane; e < p; e += 64) {
      double v;
      if (e < 12 * N) {
        const int i = e / 12, r = e % 12;
        v = (i >= 1) ? dotrow12(Md + 12 * r, X + 12 * (i - 1)) : 0.0;
        v += Pd[r] * X[12 * i + r];
        v += dotrow12(Nd + 12 * r, X + 12 * N + 12 * i);
      } else {
        const int i = (e - 12 * N) / 2, w = (e - 12 * N) % 2;
        v = SG[6 + w] * X[12 * N + 12 * i + (w ? 9 : 6)];
      }
      RE[e] = v - bg[e];
    }
    double sz = 0.0;
    for (int q = lane; q < m; q += 64) {
      const int i = q / 16, k = q % 16;
      const double v = dotrow12(Gd + 12 * k, X + 12 * N + 12 * i);
      RS[q] = (v + S[q]) - hg[q];
      sz += S[q] * Z[q];
    }
    __syncthreads();
    return wave_sum(sz) / m;
  }

  // -------------------------------------------------------------------- factorise ----
  __device__ void factor() {
    for (int q = lane; q < m; q += 64) {
      const double w = (1.0 / S[q]) * Z[q] + kDelta;
      WD[q] = w;
      DI[q] = 1.0 / (1.0 + kDelta * w);
    }
    __syncthreads();
    for (int task = lane; task < 2 * N; task += 64) {  // foot blocks of Phi_u
      const int i = task >> 1, f = task & 1;
      double a[10];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c <= r; ++c) a[r * (r + 1) / 2 + c] = (r == c) ? Hu[c_tab.foot_col[f][r]] + kBeta : 0.0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int q = 16 * i + 8 * f + k;
        const double lam = DI[q] * WD[q];
        double g4[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) g4[b] = Gd[(8 * f + k) * 12 + c_tab.foot_col[f][b]];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c <= r; ++c) a[r * (r + 1) / 2 + c] += lam * g4[r] * g4[c];
      }
      sweep_inverse<4>(a);
#pragma unroll
      for (int e = 0; e < 10; ++e) PH[20 * i + 10 * f + e] = a[e];
    }
    __syncthreads();
    for (int e = lane; e < 78 * N; e += 64) {  // S_ii = K + sum_f N_f Phi_f^-1 N_f^T
      const int i = e / 78, l = e % 78;
      int r, c;
      tri_rc(l, r, c);
      double v = (i == 0 ? K0 : K1)[l];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const double* ph = PH + 20 * i + 10 * f;
        double vc[4], vr[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          vr[a] = Nd[r * 12 + c_tab.foot_col[f][a]];
          vc[a] = Nd[c * 12 + c_tab.foot_col[f][a]];
        }
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          double t = 0.0;
#pragma unroll
          for (int b = 0; b < 4; ++b) t += ph[sym_idx(a, b)] * vc[b];
          v += vr[a] * t;
        }
      }
      DV[e] = v;
    }
    __syncthreads();
    int r0, c0, r1 = 0, c1 = 0;
    const int e0 = lane, e1 = lane + 64;
    tri_rc(e0 < 78 ? e0 : 0, r0, c0);
    if (e1 < 78) tri_rc(e1, r1, c1);
    for (int i = 0; i < N; ++i) {
      double* Di = DV + 78 * i;
      if (i >= 1) {  // D_i = S_ii - C D_{i-1}^-1 C^T
        const double* Dp = DV + 78 * (i - 1);
        for (int e = lane; e < 144; e += 64) {
          const int r = e / 12, c = e % 12;
          double u = 0.0;
#pragma unroll
          for (int k = 0; k < 12; ++k) u += Cd[r * 12 + k] * Dp[sym_idx(k, c)];
          SC[e] = u;
        }
        __syncthreads();
        for (int e = lane; e < 78; e += 64) {
          int r, c;
          tri_rc(e, r, c);
          Di[e] -= dotrow12(SC + 12 * r, Cd + 12 * c);
        }
        __syncthreads();
      }
      for (int k = 0; k < 12; ++k) {  // symmetric sweep -> -D_i^-1
        const double id = 1.0 / Di[k * (k + 1) / 2 + k];
        const double a0 = Di[e0], k0r = Di[sym_idx(r0, k)], k0c = Di[sym_idx(c0, k)];
        double a1 = 0.0, k1r = 0.0, k1c = 0.0;
        if (e1 < 78) { a1 = Di[e1]; k1r = Di[sym_idx(r1, k)]; k1c = Di[sym_idx(c1, k)]; }
        __syncthreads();
        if (e0 < 78) {
          Di[e0] = (r0 != k && c0 != k) ? a0 - k0r * k0c * id : ((r0 == k && c0 == k) ? -id : a0 * id);
        }
        if (e1 < 78) {
          Di[e1] = (r1 != k && c1 != k) ? a1 - k1r * k1c * id : ((r1 == k && c1 == k) ? -id : a1 * id);
        }
        __syncthreads();
      }
      if (e0 < 78) Di[e0] = -Di[e0];
      if (e1 < 78) Di[e1] = -Di[e1];
      __syncthreads();
    }
  }

  // ------------------------------------------------------------------------ solve ----
  // mode 0: affine rhs r2 = -(S^-1 (s o z)); mode 1: combined r2 = affine - S^-1 (s o z + ds o dz - smu)
  __device__ void solve(int mode, double smu) {
    for (int q = lane; q < m; q += 64) {
      const double si = 1.0 / S[q];
      double r2 = -(si * (S[q] * Z[q]));
      if (mode) r2 = r2 + -(si * (S[q] * Z[q] + DS[q] * DZ[q] - smu));
      VV[q] = DI[q] * (r2 + WD[q] * RS[q]);
    }
    __syncthreads();
    for (int c = lane; c < nz; c += 64) {
      double v = -RX[c];
      if (c >= 12 * N) {
        const int i = (c - 12 * N) / 12, j = (c - 12 * N) % 12;
        double g = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) g += Gd[k * 12 + j] * VV[16 * i + k];
        v -= g;
      }
      R1T[c] = v;
    }
    __syncthreads();
    for (int c = lane; c < 12 * N; c += 64) TV[c] = R1T[c] * IX[c % 12];
    for (int task = lane; task < 3 * N; task += 64) {
      if (task < 2 * N) {
        const int i = task >> 1, f = task & 1;
        const double* ph = PH + 20 * i + 10 * f;
        double rv[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) rv[a] = R1T[12 * N + 12 * i + c_tab.foot_col[f][a]];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          double t = 0.0;
#pragma unroll
          for (int b = 0; b < 4; ++b) t += ph[sym_idx(a, b)] * rv[b];
          TV[12 * N + 12 * i + c_tab.foot_col[f][a]] = t;
        }
      } else {
        const int i = task - 2 * N, b = 12 * N + 12 * i;
        const double r4a = -RE[12 * N + 2 * i], r4b = -RE[12 * N + 2 * i + 1];
        TV[b + 6] = (kDelta * R1T[b + 6] + SG[6] * r4a) / (SG[4] * kDelta + SG[6] * SG[6]);
        TV[b + 9] = (kDelta * R1T[b + 9] + SG[7] * r4b) / (SG[5] * kDelta + SG[7] * SG[7]);
        TV[b + 8] = R1T[b + 8] * SG[1];
        TV[b + 11] = R1T[b + 11] * SG[3];
      }
    }
    __syncthreads();
    for (int e = lane; e < 12 * N; e += 64) {  // g = A_dyn t + re
      const int i = e / 12, r = e % 12;
      double v = (i >= 1) ? dotrow12(Md + 12 * r, TV + 12 * (i - 1)) : 0.0;
      v += Pd[r] * TV[12 * i + r];
      v += dotrow12(Nd + 12 * r, TV + 12 * N + 12 * i);
      QV[e] = v + RE[e];
    }
    __syncthreads();
    for (int i = 0; i < N; ++i) {  // forward: q_i -= C w_{i-1}; w_i = D_i^-1 q_i
      if (i >= 1) {
        if (lane < 12) QV[12 * i + lane] -= dotrow12(Cd + 12 * lane, WV + 12 * (i - 1));
        __syncthreads();
      }
      if (lane < 12) {
        const double* Di = DV + 78 * i;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 12; ++k) acc += Di[sym_idx(lane, k)] * QV[12 * i + k];
        WV[12 * i + lane] = acc;
      }
      __syncthreads();
    }
    if (lane < 12) QV[12 * (N - 1) + lane] = WV[12 * (N - 1) + lane];
    __syncthreads();
    for (int i = N - 2; i >= 0; --i) {  // backward: y_i = w_i - D_i^-1 C^T y_{i+1}
      if (lane < 12) SC[lane] = dotcol12(Cd, lane, QV + 12 * (i + 1));
      __syncthreads();
      if (lane < 12) {
        const double* Di = DV + 78 * i;
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 12; ++k) acc += Di[sym_idx(lane, k)] * SC[k];
        QV[12 * i + lane] = WV[12 * i + lane] - acc;
      }
      __syncthreads();
    }
    for (int c = lane; c < 12 * N; c += 64) {  // dx (x part) = t - phi_x^-1 A^T dy
      const int k = c / 12 + 1, j = c % 12;
      double aty = Pd[j] * QV[12 * (k - 1) + j];
      if (k < N) aty += dotcol12(Md, j, QV + 12 * k);
      TV[c] = TV[c] - aty * IX[j];
    }
    for (int task = lane; task < 3 * N; task += 64) {
      const bool foot = task < 2 * N;
      const int i = foot ? (task >> 1) : task - 2 * N;
      const int b = 12 * N + 12 * i;
      const double* yi = QV + 12 * i;
      if (foot) {
        const int f = task & 1;
        const double* ph = PH + 20 * i + 10 * f;
        double av[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) av[a] = dotcol12(Nd, c_tab.foot_col[f][a], yi);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          double t = 0.0;
#pragma unroll
          for (int q = 0; q < 4; ++q) t += ph[sym_idx(a, q)] * av[q];
          TV[b + c_tab.foot_col[f][a]] -= t;
        }
      } else {
        const double r4a = -RE[12 * N + 2 * i], r4b = -RE[12 * N + 2 * i + 1];
        const double a6 = dotcol12(Nd, 6, yi), a9 = dotcol12(Nd, 9, yi);
        const double a8 = dotcol12(Nd, 8, yi), a11 = dotcol12(Nd, 11, yi);
        TV[b + 6] -= SG[0] * a6;
        TV[b + 9] -= SG[2] * a9;
        TV[b + 8] -= SG[1] * a8;
        TV[b + 11] -= SG[3] * a11;
        const double rho6 = R1T[b + 6] - a6, rho9 = R1T[b + 9] - a9;
        DY[12 * N + 2 * i] = (SG[6] * rho6 - SG[4] * r4a) / (SG[4] * kDelta + SG[6] * SG[6]);
        DY[12 * N + 2 * i + 1] = (SG[7] * rho9 - SG[5] * r4b) / (SG[5] * kDelta + SG[7] * SG[7]);
      }
    }
    for (int e = lane; e < 12 * N; e += 64) DY[e] = QV[e];
    __syncthreads();
    for (int q = lane; q < m; q += 64) {  // dz, ds
      const int i = q / 16, k = q % 16;
      const double gd = dotrow12(Gd + 12 * k, TV + 12 * N + 12 * i);
      const double dz = VV[q] + DI[q] * WD[q] * gd;
      DZ[q] = dz;
      DS[q] = -RS[q] - gd + kDelta * dz;
    }
    __syncthreads();
  }

  __device__ double step_length(const double* v, const double* dv) const {
    double mn = INFINITY;
    for (int q = lane; q < m; q += 64) {
      const bool c = dv[q] < 0.0;
      const double a = -v[q] / dv[q];
      mn = fmin(mn, (c ? a : 0.0) + (!c ? 1.0 : 0.0));
    }
    mn = wave_min(mn);
    return fmax(fmin(1.0, 0.99 * mn), 1e-12);
  }
};

__global__ __launch_bounds__(64) void pdipm_srbd_kernel(SolverArgs args) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int env = blockIdx.x;
  if (env >= args.batch) return;
  const int N = args.N, lane = threadIdx.x;
  const FastLayout Lo(N);
  FastCtx C;
  C.N = N; C.nz = 24 * N; C.m = 16 * N; C.p = 14 * N; C.lane = lane;
  C.Md = smem + Lo.Md; C.Nd = smem + Lo.Nd; C.Cd = smem + Lo.Cd; C.Gd = smem + Lo.Gd;
  C.K0 = smem + Lo.K0; C.K1 = smem + Lo.K1; C.Pd = smem + Lo.Pd; C.IX = smem + Lo.IX;
  C.Hu = smem + Lo.Hu; C.SG = smem + Lo.SG; C.PH = smem + Lo.PH; C.DV = smem + Lo.DV;
  C.X = smem + Lo.X; C.S = smem + Lo.S; C.Z = smem + Lo.Z; C.Y = smem + Lo.Y;
  C.RX = smem + Lo.RX; C.RS = smem + Lo.RS; C.RE = smem + Lo.RE; C.WD = smem + Lo.WD; C.DI = smem + Lo.DI;
  C.VV = smem + Lo.VV; C.R1T = smem + Lo.R1T; C.TV = smem + Lo.TV; C.QV = smem + Lo.QV; C.WV = smem + Lo.WV;
  C.DS = smem + Lo.DS; C.DZ = smem + Lo.DZ; C.DY = smem + Lo.DY; C.SC = smem + Lo.SC;
  const int nz = C.nz, m = C.m, p = C.p, nA = nnz_A(N), nG = 28 * N;
  const double* Hg = solver_in(args, 0) + (size_t)env * nz;
  const double* Gg = solver_in(args, 1) + (size_t)env * nG;
  const double* Ag = solver_in(args, 2) + (size_t)env * nA;
  C.fg = solver_in(args, 3) + (size_t)env * nz;
  C.hg = solver_in(args, 4) + (size_t)env * m;
  C.bg = solver_in(args, 5) + (size_t)env * p;

  // ---- compact load: stage-0/1 slices in dense form ----
  for (int e = lane; e < 144; e += 64) {
    const int r = e / 12, j = e % 12;
    const int om = c_tab.Mi[r][j], on = c_tab.Ni[r][j];
    C.Md[e] = (N >= 2 && om >= 0) ? Ag[a_xblock(1) + om] : 0.0;
    C.Nd[e] = on >= 0 ? Ag[a_ublock(N, 0) + on] : 0.0;
  }
  for (int e = lane; e < 192; e += 64) C.Gd[e] = 0.0;
  if (lane < 12) {
    C.Pd[lane] = Ag[a_pidx(c_tab, N, 0, lane)];
    C.Hu[lane] = Hg[12 * N + lane];
    C.Hu[12 + lane] = Hg[lane];
  }
  __syncthreads();
  if (lane < 28) C.Gd[c_tab.grow[lane] * 12 + c_tab.gcol[lane]] = Gg[lane];
  // ---- stage-invariance check (bitwise) ----
  bool bad = false;
  for (int e = lane; e < nA; e += 64) {
    double ref;
    // locate e: x blocks, x_N singles, u blocks
    if (e < 36 * (N - 1)) {
      const int loc = e % 36;
      int j = 11;
      while (c_tab.cpx[j] > loc) --j;
      const int t = loc - c_tab.cpx[j];
      ref = (t == 0) ? C.Pd[j] : C.Md[c_tab.sx[j][t - 1] * 12 + j];
    } else if (e < a_ubase(N)) {
      ref = C.Pd[e - 36 * (N - 1)];
    } else {
      const int loc = (e - a_ubase(N)) % 86;
      int j = 11;
      while (c_tab.cpu[j] > loc) --j;
      const int t = loc - c_tab.cpu[j];
      ref = (t < c_tab.su_n[j]) ? C.Nd[c_tab.su[j][t] * 12 + j] : Ag[a_ubase(N) + loc];
    }
    bad |= !(Ag[e] == ref);
  }
  for (int e = lane; e < nG; e += 64) bad |= !(Gg[e] == Gg[e % 28]);
  for (int e = lane; e < nz; e += 64) bad |= !(Hg[e] == Hg[(e < 12 * N ? 0 : 12 * N) + e % 12]);
  const bool any_bad = __any(bad);
  if (any_bad) {
    if (lane == 0) {
      double* mo = solver_out(args, 5) + (size_t)env;
      *mo = __longlong_as_double((long long)kFallbackBits);
    }
    return;
  }
  // ---- per-QP constants ----
  if (lane < 12) C.IX[lane] = 1.0 / (C.Hu[12 + lane] + kBeta);
  if (lane == 0) {
    const double e6 = Ag[a_ubase(N) + c_tab.e6], e9 = Ag[a_ubase(N) + c_tab.e9];
    const double p6 = C.Hu[6] + kBeta, p9 = C.Hu[9] + kBeta;
    C.SG[0] = kDelta / (p6 * kDelta + e6 * e6);
    C.SG[1] = 1.0 / (C.Hu[8] + kBeta);
    C.SG[2] = kDelta / (p9 * kDelta + e9 * e9);
    C.SG[3] = 1.0 / (C.Hu[11] + kBeta);
    C.SG[4] = p6;
    C.SG[5] = p9;
    C.SG[6] = e6;
    C.SG[7] = e9;
  }
  __syncthreads();
  for (int e = lane; e < 144; e += 64) {
    const int r = e / 12, j = e % 12;
    C.Cd[e] = C.Md[e] * (C.Pd[j] * C.IX[j]);
  }
  for (int e = lane; e < 78; e += 64) {
    int r, c;
    tri_rc(e, r, c);
    double k0 = (r == c) ? C.Pd[r] * C.Pd[r] * C.IX[r] + kDelta : 0.0;
    k0 += C.Nd[r * 12 + 6] * C.Nd[c * 12 + 6] * C.SG[0] + C.Nd[r * 12 + 8] * C.Nd[c * 12 + 8] * C.SG[1] +
          C.Nd[r * 12 + 9] * C.Nd[c * 12 + 9] * C.SG[2] + C.Nd[r * 12 + 11] * C.Nd[c * 12 + 11] * C.SG[3];
    double k1 = k0;
#pragma unroll
    for (int j = 0; j < 12; ++j) k1 += C.Md[r * 12 + j] * C.Md[c * 12 + j] * C.IX[j];
    C.K0[e] = k0;
    C.K1[e] = k1;
  }
  // ---- iterate ----
  if (args.init_mode == 0) {
    const double* xg = solver_in(args, 6) + (size_t)env * nz;
    const double* sg = solver_in(args, 7) + (size_t)env * m;
    const double* zg = solver_in(args, 8) + (size_t)env * m;
    const double* yg = solver_in(args, 9) + (size_t)env * p;
    for (int e = lane; e < nz; e += 64) C.X[e] = xg[e];
    for (int e = lane; e < m; e += 64) { C.S[e] = sg[e]; C.Z[e] = zg[e]; }
    for (int e = lane; e < p; e += 64) C.Y[e] = yg[e];
  } else {
    for (int e = lane; e < nz; e += 64) C.X[e] = 0.0;
    for (int e = lane; e < m; e += 64) { C.S[e] = fmax(C.hg[e] - 0.0, 1.0); C.Z[e] = 1.0; }
    for (int e = lane; e < p; e += 64) C.Y[e] = args.y0;
  }
  __syncthreads();

  double res0 = 0.0, res1 = 0.0, res2 = 0.0, mu_new = 0.0;
  for (int it = 0; it < args.n_iter; ++it) {
    const double mu = C.residuals();
    C.factor();
    C.solve(0, 0.0);
    const double ap = C.step_length(C.S, C.DS), ad = C.step_length(C.Z, C.DZ);
    double sza = 0.0;
    for (int q = lane; q < m; q += 64) sza += (C.S[q] + ap * C.DS[q]) * (C.Z[q] + ad * C.DZ[q]);
    const double mu_aff = wave_sum(sza) / m;
    const double sigma = pow(mu_aff / mu, 3.0);
    __syncthreads();
    C.solve(1, sigma * mu * 1.0);
    const double apc = C.step_length(C.S, C.DS), adc = C.step_length(C.Z, C.DZ);
    __syncthreads();
    double szn = 0.0;
    for (int e = lane; e < nz; e += 64) C.X[e] = C.X[e] + apc * C.TV[e];
    for (int q = lane; q < m; q += 64) {
      const double sn = fmax(C.S[q] + apc * C.DS[q], 1e-8);
      const double zn = fmax(fmax(C.Z[q] + adc * C.DZ[q], 1e-8), 1e-8);
      C.S[q] = sn;
      C.Z[q] = zn;
      szn += sn * zn;
    }
    for (int e = lane; e < p; e += 64) C.Y[e] = C.Y[e] + adc * C.DY[e];
    mu_new = wave_sum(szn) / m;
    if (it == args.n_iter - 1) {
      double a = 0.0, b = 0.0, c = 0.0;
      for (int e = lane; e < nz; e += 64) a += C.RX[e] * C.RX[e];
      for (int e = lane; e < m; e += 64) b += C.RS[e] * C.RS[e];
      for (int e = lane; e < p; e += 64) c += C.RE[e] * C.RE[e];
      res0 = sqrt(wave_sum(a));
      res1 = sqrt(wave_sum(b));
      res2 = sqrt(wave_sum(c));
    }
    __syncthreads();
  }
  double* xo = solver_out(args, 0) + (size_t)env * nz;
  double* so = solver_out(args, 1) + (size_t)env * m;
  double* zo = solver_out(args, 2) + (size_t)env * m;
  double* yo = solver_out(args, 3) + (size_t)env * p;
  double* ro = solver_out(args, 4) + (size_t)env * 4;
  double* mo = solver_out(args, 5) + (size_t)env;
  for (int e = lane; e < nz; e += 64) xo[e] = C.X[e];
  for (int e = lane; e < m; e += 64) { so[e] = C.S[e]; zo[e] = C.Z[e]; }
  for (int e = lane; e < p; e += 64) yo[e] = C.Y[e];
  if (lane == 0) {
    ro[0] = res0;
    ro[1] = res1;
    ro[2] = res2;
    ro[3] = mu_new;
    mo[0] = mu_new;
  }
}

}  // namespace srbd
