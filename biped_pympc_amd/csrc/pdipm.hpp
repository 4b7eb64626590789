// pdipm.hpp -- HIP kernel for the batched Mehrotra primal-dual interior-point Newton loop.
//
// Replaces the CusADi-generated kernel of CasADi Function 'sparse_pdipm_multiple_iterations'
// (reference biped_pympc/casadi/sparse_pdipm_solver.py:357-534), same 10 inputs / 6 outputs and
// the same batched row layout, but with the Newton-iteration count a RUNTIME argument (the
// reference bakes 5 iterations into a ~3 h compile, README.md:80-84).
//
// Per iteration the reference factorises the full 70N x 70N quasi-definite KKT
//   [[H+bI, 0, G^T, A^T], [0, S^-1Z+dI, I, 0], [G, I, -dI, 0], [A, 0, 0, -dI]]
// with a sparse LDL^T and solves it twice (affine + corrector). This kernel solves the SAME linear
// systems by exact block elimination, exploiting the stage structure:
//   W = S^-1 Z + dI, D = I + dW, Lam = D^-1 W            (diagonal)
//   dz = D^-1 (r2 - W r3) + Lam G dx,   ds = r3 - G dx + d dz
//   [[Phi, A^T], [A, -dI]] [dx; dy] = [r1 - G^T D^-1 (r2 - W r3); r4],  Phi = H + bI + G^T Lam G
// Phi is block diagonal per stage (x: diagonal; u: two 4x4 foot blocks + 4 scalars). The two
// x-moment rows per stage pair with the decoupled u_i[6], u_i[9] and are eliminated as exact 2x2
// blocks, leaving the dual system (A_dyn Phi^-1 A_dyn^T + dI) dy = g, which is block-tridiagonal
// with 12x12 SPD blocks. It is factored by a block recursion D_i = S_ii - S_{i,i-1} D_{i-1}^-1
// S_{i,i-1}^T keeping explicit D_i^-1 (symmetric sweep), and the corrector reuses the factors
// (as the reference reuses its LDL, :482). Affine and corrector right-hand sides are combined
// into one solve (linear, so identical in exact arithmetic).
//
// Mapping (gfx950): one wavefront per QP; the QP's CCS values (H, G, A), its iterate and all
// factors live in LDS for the whole solve (loaded once, coalesced); f, h, b are re-read from
// global each iteration (L2-resident). Stage-parallel work (residuals, Phi blocks, the N
// diagonal dual blocks) is spread over the 64 lanes; the stage recursion is sequential.
#pragma once
#include "srbd_common.hpp"
#include "dpp_rows.hpp"

namespace srbd {

struct SolverArgs {
  const double* in[10];  // Q_val, G_val, A_val, f, h, b, x, s, z, y
  double* out[6];        // x, s, z, y, residuals(4), mu(1)
  const double* const* dev_in;
  double* const* dev_out;
  int N;
  int n_iter;
  int batch;
  int init_mode;  // 0: iterate from inputs 6..9; 1: x=0, s=max(h,1), z=1, y=y0 (GPU caller init);
                  // 2: x = input 6, s = max(h - G x, 1), z = 1, y = 0 (_ccs init)
  double y0;
  // the library's per-device pool for QPs the stage-invariant kernels cannot take: scratch_slots
  // slots of scratch_stride doubles, each guarded by a lock word (0 = free) at
  // scratch_locks[slot * kLockStride] (one 128-byte line per lock: no false sharing between slots)
  double* scratch;
  int* scratch_locks;
  int scratch_slots;
  int scratch_stride;  // doubles per slot: the largest SolverLayout(N).total over N = 1..kMaxN
  int* status;  // (batch) per-problem status word (kStatus* bits), or null: not written
  int refine_policy;  // the register kernels' refinement policy word (srbd_set_refinement_policy)
  double refine_w;    // its W = z / s vote threshold (INFINITY: no W vote)
};

// Refinement policy word of the register kernels (include/srbd_mpc.h SRBD_REFINE_*): bit 0 the affine
// direction in every iteration, bit 1 at an iterate whose duals z are all 1 (a solve's initial iterate), bits
// 8-15 / 16-23 in the first / last k iterations
constexpr int kRefineAffineAll = 1, kRefineAffineAtInit = 2;

// Per-problem status word (SURVEY.md 5 "failure detection"; the reference has only its clamps,
// sparse_pdipm_solver.py:466-467,501-515): bit 0 a non-finite value in the returned x, s, z, y or
// mu; bit 1 a combined-direction step length (primal or dual) at its 1e-12 floor in the last
// iteration; bit 2 the QP was not stage-invariant and took the general solve (scratch fallback).
constexpr int kStatusNonFinite = 1, kStatusStepFloor = 2, kStatusFallback = 4;
constexpr int kLockStride = 32;  // ints between two slots' lock words
__device__ __forceinline__ bool not_finite(double v) { return !__builtin_isfinite(v); }

// iterative-refinement steps per direction in the LDS-resident and general kernels (the register
// kernels' one step sits at the FP64 floor at N = 10 / 20)
constexpr int kRefineSteps = 1;

// threads per QP in the general kernel (pdipm_kernel): two waves share its row-parallel loops (the
// chains run on the first wave's 32 lanes); at ~410 VGPRs each wave has a SIMD to itself, and the two
// QPs per CU its LDS allows at N = 10 then use all four SIMDs
constexpr int kGeneralThreads = 128;


__device__ inline const double* solver_in(const SolverArgs& a, int i) {
  return a.dev_in ? a.dev_in[i] : a.in[i];
}
__device__ inline double* solver_out(const SolverArgs& a, int i) {
  return a.dev_out ? a.dev_out[i] : a.out[i];
}

constexpr int kTablesDoubles = (int)((sizeof(Tables) + 15) / 16) * 2;
// the same tables as a compile-time constant: lookups at indices known after unrolling fold away
constexpr Tables kTabs = make_tables();

// The dual coupling S_{i,i-1} = M_i diag(P_{i-1} / phi_x(x_i)) has M_i's CCS pattern, which the twisted
// chains of SolverCtx (as those of pdipm_srbd.hpp FastCtx) rely on: row c holds {c}, plus {6, 7, 8}
// for c < 3 and {c + 6} for 3 <= c < 6; and pi C^T pi^T (pi = perm12) has the same pattern, so the
// backward group runs the forward group's instructions.
// G's CCS columns are contiguous runs of at most 8 entries (gcol_dot's unrolled form)
constexpr bool g_columns_ok() {
  for (int q = 0; q < 28; ++q)
    if (q < kTabs.gcp[kTabs.gcol[q]] || q >= kTabs.gcp[kTabs.gcol[q]] + kTabs.gcn[kTabs.gcol[q]]) return false;
  for (int j = 0; j < 12; ++j)
    if (kTabs.gcn[j] > 8) return false;
  return true;
}
static_assert(g_columns_ok(), "G column runs");
// the foot rows of G: row 8 + k (right foot) has row k's (left foot) pattern, mirrored foot columns
constexpr bool g_feet_ok() {
  for (int k = 0; k < 8; ++k) {
    if (kTabs.gr_n[k] != kTabs.gr_n[8 + k]) return false;
    for (int t = 0; t < kTabs.gr_n[k]; ++t) {
      const int a = kTabs.gr_col[k][t], b = kTabs.gr_col[8 + k][t];
      if (kTabs.col_foot[a] != 0 || kTabs.col_foot[b] != 1 || kTabs.col_pos[a] != kTabs.col_pos[b]) return false;
    }
  }
  return true;
}
static_assert(g_feet_ok(), "G foot rows");

constexpr bool coupling_pattern_ok() {
  for (int r = 0; r < 12; ++r)
    for (int j = 0; j < 12; ++j) {
      const bool want = j == r || (r < 3 && j >= 6 && j <= 8) || (r >= 3 && r < 6 && j == r + 6);
      if ((kTabs.Mi[r][j] >= 0) != want || (kTabs.Mi[perm12(j)][perm12(r)] >= 0) != want) return false;
    }
  return true;
}
static_assert(coupling_pattern_ok(), "A's x-block pattern is not the one the twisted chains assume");

// LDS carve (doubles) for horizon N; every offset is a multiple of 2 doubles (16 B).
struct SolverLayout {
  int AV, GV, HV, X, S, Z, Y, RX, RS, RE, SI, WD, DI, R2, VV, PH, DV, R1T, TV, QV, WV, DS, DZ, DY, SC,
      RD, TB, CV, KX, total;
  __host__ __device__ SolverLayout(int N) {
    const int nz = 24 * N, m = 16 * N, p = 14 * N, nd = 12 * N;
    int o = 0;
    auto take = [&](int n) { int r = o; o += (n + 1) & ~1; return r; };
    AV = take(122 * N - 24); GV = take(28 * N); HV = take(nz);
    X = take(nz); S = take(m); Z = take(m); Y = take(p);
    RX = take(nz); RS = take(m); RE = take(p);
    SI = take(m); WD = take(m); DI = take(m); R2 = take(m); VV = take(m);
    PH = take(24 * N); DV = take(78 * N);
    R1T = take(nz); TV = take(nz);
    QV = take(nd); WV = take(nd);
    DS = take(m); DZ = take(m); DY = take(p);
    SC = take(448);  // 2 x 144 V scratch + 144 middle block + 12 middle vector (the twisted chains)
    RD = take(8);    // the team reductions' wave partials
    TB = take(kTablesDoubles);  // a copy of c_tab: the index tables, read with lane-varying indices
    // the dual couplings S_{i,i-1} = M_i diag(P_{i-1} / phi_x(x_i)) over x_i's 36-value block (cpl), where
    // they still fit the 160 KiB of LDS a workgroup may have (all horizons but 32; else formed on the fly)
    CV = (o + 36 * N) * 8 <= 160 * 1024 ? take(36 * N) : -1;
    // the constant x part of every S_ii (sii_x; the general kernel only), where it still fits
    KX = (CV >= 0 && (o + 78 * N) * 8 <= 160 * 1024) ? take(78 * N) : -1;
    total = o;
  }
};

__device__ inline int sym_idx(int a, int b) { return a >= b ? a * (a + 1) / 2 + b : b * (b + 1) / 2 + a; }

// Symmetric sweep of a small SPD matrix held in registers (packed lower) -> its inverse.
// kRcp: pivot reciprocals by rcp3 instead of IEEE division.
template <int n, bool kRcp = false>
__device__ inline void sweep_inverse(double (&a)[n * (n + 1) / 2]) {
#pragma unroll
  for (int k = 0; k < n; ++k) {
    const double id = kRcp ? rcp3(a[k * (k + 1) / 2 + k]) : 1.0 / a[k * (k + 1) / 2 + k];
    double col[n];
#pragma unroll
    for (int i = 0; i < n; ++i) col[i] = a[sym_idx(i, k)];
#pragma unroll
    for (int r = 0; r < n; ++r)
#pragma unroll
      for (int c = 0; c <= r; ++c) {
        const int e = r * (r + 1) / 2 + c;
        if (r != k && c != k) a[e] = a[e] - col[r] * col[c] * id;
        else if (r == k && c == k) a[e] = -id;
        else a[e] = a[e] * id;
      }
  }
#pragma unroll
  for (int e = 0; e < n * (n + 1) / 2; ++e) a[e] = -a[e];
}

// LDL^T of a packed symmetric positive definite block (lower packed, sym_idx order), no pivoting
// (backward stable for SPD): on return the diagonal slots hold 1 / d_j, the others L_ij. Used where a
// solve must keep the stiff direction: Phi_f reaches cond ~1e12 as the barrier sharpens, and an
// explicit inverse applied to a vector loses the component along G_i (error ~cond x that of a stable
// solve) that Lambda ~ W then multiplies into dz (scripts/stiff_dz_emu.py).
// kRcp: pivot reciprocals by rcp3 (v_rcp_f64 + the cubic step, correctly rounded; the register kernels'
// hot loop) instead of IEEE division (the general and LDS-resident kernels).
template <int n, bool kRcp = false>
__device__ inline void ldlt_factor(double (&a)[n * (n + 1) / 2]) {
  double d[n];
#pragma unroll
  for (int j = 0; j < n; ++j) {
    double dj = a[j * (j + 1) / 2 + j];
#pragma unroll
    for (int k = 0; k < j; ++k) dj -= a[j * (j + 1) / 2 + k] * a[j * (j + 1) / 2 + k] * d[k];
    d[j] = dj;
    const double id = kRcp ? rcp3(dj) : 1.0 / dj;
#pragma unroll
    for (int i = j + 1; i < n; ++i) {
      double v = a[i * (i + 1) / 2 + j];
#pragma unroll
      for (int k = 0; k < j; ++k) v -= a[i * (i + 1) / 2 + k] * a[j * (j + 1) / 2 + k] * d[k];
      a[i * (i + 1) / 2 + j] = v * id;
    }
    a[j * (j + 1) / 2 + j] = id;
  }
}
// x = A^-1 v from ldlt_factor's packed factors at f (LDS or registers)
template <int n>
__device__ inline void ldlt_solve_p(const double* f, const double (&v)[n], double (&x)[n]) {
#pragma unroll
  for (int i = 0; i < n; ++i) {
    double y = v[i];
#pragma unroll
    for (int k = 0; k < i; ++k) y -= f[i * (i + 1) / 2 + k] * x[k];
    x[i] = y;
  }
#pragma unroll
  for (int i = 0; i < n; ++i) x[i] *= f[i * (i + 1) / 2 + i];
#pragma unroll
  for (int i = n - 1; i >= 0; --i) {
#pragma unroll
    for (int k = i + 1; k < n; ++k) x[i] -= f[k * (k + 1) / 2 + i] * x[k];
  }
}
template <int n>
__device__ inline void ldlt_solve(const double (&f)[n * (n + 1) / 2], const double (&v)[n], double (&x)[n]) {
#pragma unroll
  for (int i = 0; i < n; ++i) {
    double y = v[i];
#pragma unroll
    for (int k = 0; k < i; ++k) y -= f[i * (i + 1) / 2 + k] * x[k];
    x[i] = y;
  }
#pragma unroll
  for (int i = 0; i < n; ++i) x[i] *= f[i * (i + 1) / 2 + i];
#pragma unroll
  for (int i = n - 1; i >= 0; --i) {
#pragma unroll
    for (int k = i + 1; k < n; ++k) x[i] -= f[k * (k + 1) / 2 + i] * x[k];
  }
}

// (G x)_q of inequality row q from the stage's 28 CCS values of G (c_tab.grow / gcol) and the u
// part xu of x, each product rounded: the reference's G_mat @ x_init (sparse_pdipm_solver.py:31);
// a row holds at most two nonzeros, so every summation order gives this value.
__device__ inline double ccs_gx(const double* Gv, int q, const double* xu) {
#pragma clang fp contract(off)
  const int i = q / 16, k = q % 16;
  double acc = 0.0;
  for (int t = 0; t < 28; ++t)
    if (c_tab.grow[t] == k) acc += Gv[28 * i + t] * xu[12 * i + c_tab.gcol[t]];
  return acc;
}

// A call to one phase of the general solve: inlined into the general kernel (kInl: the whole solve is
// one function, so its working set is known to be LDS -- ds_read / ds_write -- instead of flat accesses
// through a context object kept in scratch: 1,059 flat loads and 247 scratch accesses before), a real
// call in the in-launch fallback of the stage-invariant kernels (inlined there, the solve would need
// ~370 VGPRs under their 256-register budget and clobber every VGPR across the call).
#define SRBD_GCALL(...)                          \
  do {                                           \
    if constexpr (kInl) {                        \
      [[clang::always_inline]] __VA_ARGS__;      \
    } else {                                     \
      __VA_ARGS__;                               \
    }                                            \
  } while (0)

struct SolverCtx {
  int N, nz, m, p, nd, lane;
  // nt: the threads a QP's row-parallel loops stride over (kGeneralThreads in the general kernel; in
  // the fallback the calling kernel's threads per QP: 64, 128, 192 or 256); RD: one partial per wave
  int nt;
  double* RD;
  double *AV, *GV, *HV, *X, *S, *Z, *Y, *RX, *RS, *RE, *SI, *WD, *DI, *R2, *VV, *PH, *DV, *R1T, *TV,
      *QV, *WV, *DS, *DZ, *DY, *SC;
  const double *fg, *hg, *bg;
  double *xsg, *ysg;  // this QP's x / y output rows: the saved dx / dy during the refinement solve
  // the index tables (a copy of c_tab in LDS where one fits: its lookups take lane-varying indices,
  // which from constant memory are vector loads of L2 latency on every chain step) and the couplings
  double* CV;
  double* KX;  // sii_x of every stage (packed lower, 78 per stage), or null: formed in factor()
  const Tables* T;
  PROF_DECL  // diagnostic phase stamps (scripts/general_phase_profile.py); empty in the product build

  // ---- structured access to the CCS values (stage-periodic tables) ----
  __device__ double Pv(int i, int r) const { return AV[a_pidx(*T, N, i, r)]; }
  __device__ double Mv(int i, int r, int j) const {  // stage i rows x x_i columns, i >= 1
    const int o = T->Mi[r][j];
    return o >= 0 ? AV[a_xblock(i) + o] : 0.0;
  }
  __device__ double Nv(int i, int r, int j) const {
    const int o = T->Ni[r][j];
    return o >= 0 ? AV[a_ublock(N, i) + o] : 0.0;
  }
  __device__ double E6(int i) const { return AV[a_ublock(N, i) + kTabs.e6]; }
  __device__ double E9(int i) const { return AV[a_ublock(N, i) + kTabs.e9]; }
  // acc += sum over the G entries of u column j of stage i (CCS order: the column's contiguous run
  // gcp[j] .. + gcn[j]) of value * v[stage-local row]: the at most 8 entries unrolled with clamped
  // indices, no branch (the sparse sums below likewise add their entries in order)
  __device__ void gcol_dot(int i, int j, const double* v, double& acc) const {
    const int b = T->gcp[j], n = T->gcn[j];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int q = b + (t < n ? t : 0);
      const double p_ = G(i, q) * v[T->grow[q]];
      acc += t < n ? p_ : 0.0;
    }
  }
  // s + (G_i xu)_k over inequality row k's entries (at most two)
  __device__ double grow_dot(int i, int k, const double* xu, double s) const {
    const int n = T->gr_n[k];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int tt = t < n ? t : 0;
      const double p_ = G(i, T->gr_off[k][tt]) * xu[T->gr_col[k][tt]];
      s += t < n ? p_ : 0.0;
    }
    return s;
  }
  // s + sum_t AV[b + t] * v[idx[t]] over the n <= NMAX entries of a CCS column
  template <int NMAX>
  __device__ double col_dot(int b, int n, const int8_t* idx, const double* v, double s) const {
#pragma unroll
    for (int t = 0; t < NMAX; ++t) {
      const int tt = t < n ? t : 0;
      const double p_ = AV[b + tt] * v[idx[tt]];
      s += t < n ? p_ : 0.0;
    }
    return s;
  }
  __device__ double phix(int k, int j) const { return HV[12 * (k - 1) + j] + kBeta; }  // x_k, k >= 1
  __device__ double phiu(int i, int j) const { return HV[12 * N + 12 * i + j] + kBeta; }
  // (M_i v)_r and (N_i v)_r of stage i (v: 12 entries), branch-free
  __device__ double mrow(int i, int r, const double* v) const {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const int o = T->Mi[r][j];
      s += (o >= 0 ? AV[a_xblock(i) + (o >= 0 ? o : 0)] : 0.0) * v[j];
    }
    return s;
  }
  __device__ double nrow(int i, int r, const double* v) const {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const int o = T->Ni[r][j];
      s += (o >= 0 ? AV[a_ublock(N, i) + (o >= 0 ? o : 0)] : 0.0) * v[j];
    }
    return s;
  }
  // The x part of S_ii (entry (r, c), r >= c): P_i^2 / phi_x(x_{i+1}) + delta on the diagonal plus
  // sum_j M_i[r][j] M_i[c][j] / phi_x(x_i)[j] -- constant over the Newton iterations
  __device__ double sii_x(int i, int r, int c) const {
    double v = 0.0;
    if (r == c) {
      const double pr = Pv(i, r);
      v = pr * pr / phix(i + 1, r) + kDelta;
    }
    if (i >= 1)
#pragma unroll
      for (int j = 0; j < 12; ++j) {
        const int o1 = T->Mi[r][j], o2 = T->Mi[c][j];
        const bool nz = o1 >= 0 && o2 >= 0;
        const double t = AV[a_xblock(i) + (nz ? o1 : 0)] * AV[a_xblock(i) + (nz ? o2 : 0)] / phix(i, j);
        v += nz ? t : 0.0;
      }
    return v;
  }
  // CV / KX: the QP's constant couplings and S_ii x parts (H and A do not change across the Newton
  // iterations); kK: KX is in use (the general kernel)
  template <bool kK>
  __device__ void couplings() {
    if (CV)
      for (int e = lane; e < 36 * (N - 1); e += nt) {
        const int i = e / 36 + 1, o = e % 36, j = T->xb_j[o];
        CV[e] = T->xb_r[o] >= 0 ? AV[a_xblock(i) + o] * Pv(i - 1, j) / phix(i, j) : 0.0;
      }
    if constexpr (kK) {
      if (KX)
        for (int e = lane; e < 78 * N; e += nt) {
          const int i = e / 78, l = e % 78;
          int r = 0;
          while ((r + 1) * (r + 2) / 2 <= l) ++r;
          KX[e] = sii_x(i, r, l - r * (r + 1) / 2);
        }
    }
  }
  __device__ double G(int i, int q) const { return GV[28 * i + q]; }
  // sum / min over the team (wave partials combined in wave order; one wave: wave_sum / wave_min)
  template <bool kMin>
  __device__ double team_reduce(double v) const {
    v = kMin ? wave_min(v) : wave_sum(v);
    if (nt == 64) return v;
    __syncthreads();  // the previous reduction's reads of RD are done
    if ((lane & 63) == 0) RD[lane >> 6] = v;
    __syncthreads();
    double r = RD[0];
    for (int w = 1; w < nt / 64; ++w) r = kMin ? fmin(r, RD[w]) : r + RD[w];
    return r;
  }
  __device__ double team_sum(double v) const { return team_reduce<false>(v); }
  __device__ double team_min(double v) const { return team_reduce<true>(v); }
  // S_{i,i-1} at x_i's CCS offset o (CV, or formed on the fly where CV did not fit)
  __device__ double cpl(int i, int o) const {
    if (CV) return CV[a_xblock(i) + o];
    const int j = T->xb_j[o];
    return AV[a_xblock(i) + o] * Pv(i - 1, j) / phix(i, j);
  }
  // Entry (c, b) of the coupling seen by twisted group g (pdipm_srbd.hpp FastCtx::cg, per stage):
  // C = S_{i,i-1} (g = 0) or pi C^T pi^T (g = 1). cg_off: its offset inside the x block (-1: a
  // structural zero), runtime indices from the LDS table; cgk: the value at compile-time c, b (after
  // unrolling both candidate offsets fold), `stage` the i of the S_{i,i-1} it comes from.
  __device__ int cg_off(int g, int c, int b) const { return g ? T->Mi[perm12(b)][perm12(c)] : T->Mi[c][b]; }
  __device__ double cgk(int g, int stage, int c, int b) const {
    return cpl(stage, g ? kTabs.Mi[perm12(b)][perm12(c)] : kTabs.Mi[c][b]);
  }
  __device__ double cg_at(int stage, int o) const { return o >= 0 ? cpl(stage, o) : 0.0; }

  // ---------------------------------------------------------------------- residuals ----
  // rx = Qx + f + G^T z + A^T y ; re = A x - b ; rs = G x + s - h ; returns mu = s'z/m
  __device__ double residuals() {
    for (int c = lane; c < nz; c += nt) {
      double v = HV[c] * X[c] + fg[c];
      if (c >= 12 * N) {
        const int i = (c - 12 * N) / 12, j = (c - 12 * N) % 12;
        double gz = 0.0;
        gcol_dot(i, j, Z + 16 * i, gz);
        double ay = 0.0;
        const int ub = a_ublock(N, i) + T->cpu[j];
        ay = col_dot<8>(ub, T->su_n[j], T->su[j], Y + 12 * i, ay);
        if (j == 6) ay += AV[ub + T->su_n[j]] * Y[12 * N + 2 * i];
        if (j == 9) ay += AV[ub + T->su_n[j]] * Y[12 * N + 2 * i + 1];
        v = (v + gz) + ay;
      } else {
        const int k = c / 12 + 1, j = c % 12;
        double ay;
        if (k < N) {
          const int xb = a_xblock(k) + T->cpx[j];
          ay = AV[xb] * Y[12 * (k - 1) + j];
          ay = col_dot<4>(xb + 1, T->sx_n[j], T->sx[j], Y + 12 * k, ay);
        } else {
          ay = AV[36 * (N - 1) + j] * Y[12 * (k - 1) + j];
        }
        v = v + ay;
      }
      RX[c] = v;
    }
    for (int e = lane; e < p; e += nt) {
      double v = 0.0;
      if (e < 12 * N) {
        const int i = e / 12, r = e % 12;
        if (i >= 1) v += mrow(i, r, X + 12 * (i - 1));
        v += Pv(i, r) * X[12 * i + r];
        v += nrow(i, r, X + 12 * N + 12 * i);
      } else {
        const int i = (e - 12 * N) / 2, w = (e - 12 * N) % 2;
        v = (w == 0 ? E6(i) * X[12 * N + 12 * i + 6] : E9(i) * X[12 * N + 12 * i + 9]);
      }
      RE[e] = v - bg[e];
    }
    double sz = 0.0;
    for (int q = lane; q < m; q += nt) {
      const int i = q / 16, k = q % 16;
      double v = 0.0;
      v = grow_dot(i, k, X + 12 * N + 12 * i, v);
      RS[q] = (v + S[q]) - hg[q];
      sz += S[q] * Z[q];
    }
    __syncthreads();
    return team_sum(sz) / m;
  }

  // ---------------------------------------------------------------------- factorise ----
  __device__ void factor() {
    for (int q = lane; q < m; q += nt) {
      const double si = 1.0 / S[q];
      const double w = si * Z[q] + kDelta;  // S^-1 Z + delta I (sparse_pdipm_solver.py:427)
      SI[q] = si;
      WD[q] = w;
      DI[q] = 1.0 / (1.0 + kDelta * w);
    }
    __syncthreads();
    // Phi_u foot blocks (lane per (stage, foot)) and decoupled scalars (lane per stage)
    for (int task = lane; task < 3 * N; task += nt) {
      if (task < 2 * N) {
      const int i = task >> 1, f = task & 1;
      double a[10];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c <= r; ++c) a[r * (r + 1) / 2 + c] = (r == c) ? phiu(i, T->foot_col[f][r]) : 0.0;
      // compile-time row patterns (the same for both feet, g_feet_ok): no table lookups, and the
      // structural zeros of each rank-1 update skipped
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int q = 16 * i + 8 * f + k;
        const double lam = DI[q] * WD[q];
        double g4[4] = {0.0, 0.0, 0.0, 0.0};
        int nzm = 0;
#pragma unroll
        for (int t = 0; t < kTabs.gr_n[k]; ++t) {
          const int pos = kTabs.col_pos[kTabs.gr_col[k][t]];
          g4[pos] = G(i, f ? kTabs.gr_off[8 + k][t] : kTabs.gr_off[k][t]);
          nzm |= 1 << pos;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c <= r; ++c)
            if ((nzm >> r) & (nzm >> c) & 1) a[r * (r + 1) / 2 + c] += lam * g4[r] * g4[c];
      }
      ldlt_factor<4>(a);  // every use of Phi_f^-1 is a stable solve with these factors
#pragma unroll
      for (int e = 0; e < 10; ++e) PH[24 * i + 10 * f + e] = a[e];
      } else {
      const int i = task - 2 * N;
      const double p6 = phiu(i, 6), p9 = phiu(i, 9), e6 = E6(i), e9 = E9(i);
      PH[24 * i + 20] = kDelta / (p6 * kDelta + e6 * e6);  // gamma_6 (exact 2x2 elimination)
      PH[24 * i + 21] = kDelta / (p9 * kDelta + e9 * e9);
      PH[24 * i + 22] = 1.0 / phiu(i, 8);
      PH[24 * i + 23] = 1.0 / phiu(i, 11);
      }
    }
    __syncthreads();
    // diagonal dual blocks S_ii (all stages in parallel), packed lower 78 per stage
    for (int e = lane; e < 78 * N; e += nt) {
      const int i = e / 78, l = e % 78;
      int r = 0;
      while ((r + 1) * (r + 2) / 2 <= l) ++r;
      const int c = l - r * (r + 1) / 2;
      double v = KX ? KX[e] : sii_x(i, r, c);
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        double vr[4], vc[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          vr[a] = Nv(i, r, T->foot_col[f][a]);
          vc[a] = Nv(i, c, T->foot_col[f][a]);
        }
        double pv[4];
        ldlt_solve_p<4>(PH + 24 * i + 10 * f, vc, pv);
#pragma unroll
        for (int a = 0; a < 4; ++a) v += vr[a] * pv[a];
      }
      v += Nv(i, r, 6) * Nv(i, c, 6) * PH[24 * i + 20] + Nv(i, r, 9) * Nv(i, c, 9) * PH[24 * i + 21] +
           Nv(i, r, 8) * Nv(i, c, 8) * PH[24 * i + 22] + Nv(i, r, 11) * Nv(i, c, 11) * PH[24 * i + 23];
      DV[e] = v;
    }
    __syncthreads();
    PROF_ADD_CTX((*this), 1);
    // Twisted block recursion (pdipm_srbd.hpp FastCtx::factor with the couplings of each stage),
    // register-resident, one block row per lane, no workgroup barrier inside:
    //   group 0 (lanes 0..15)  forward  D_i = S_ii - C_i D_{i-1}^-1 C_i^T                 i = 0 .. mid-1
    //   group 1 (lanes 16..31) backward E_j = S_jj - C_{j+1}^T E_{j+1}^-1 C_{j+1}         j = N-1 .. mid+1
    //   middle (group 0)       T = S_mm - C_m D_{m-1}^-1 C_m^T - C_{m+1}^T E_{m+1}^-1 C_{m+1}
    // with C_i = S_{i,i-1}; group 1 in pi-permuted coordinates. Each 12x12 block is inverted in
    // registers (inverse_rows12) and stored, original coordinates packed lower, in DV: D_i^-1 (i < mid),
    // T^-1 (mid), E_j^-1 (j > mid). Half the sequential steps of the one-sided recursion.
    {
      const int mid = N / 2, nf = mid, nb = N - 1 - mid;
      const int TT = nf > nb ? nf : nb;
      if (lane < 32) {
        const int g = lane >> 4;
        const int r = (lane & 15) < 12 ? (lane & 15) : 11;
        const bool own = (lane & 15) < 12;
        const int pr = g ? perm12(r) : r;
        const int cnt = g ? nb : nf;
        double* Vs = SC + 144 * g;  // per-group scratch for V = D^-1 Cg^T
        double* XB = SC + 288;      // group 1's C^T E^-1 C (permuted) for the middle block
        // offsets of row r's coupling entries: (r, r), (r, 6..8) for r < 3, (r, r + 6) for 3 <= r < 6
        const int oRR = cg_off(g, r, r);
        const int o6 = r < 3 ? cg_off(g, r, 6) : 0, o7 = r < 3 ? cg_off(g, r, 7) : 0;
        const int o8 = r < 3 ? cg_off(g, r, 8) : 0, oR6 = (r >= 3 && r < 6) ? cg_off(g, r, r + 6) : 0;
        double Dr[12];
#pragma unroll
        for (int c = 0; c < 12; ++c) Dr[c] = 0.0;
#pragma unroll 1
        for (int t = 0; t <= TT; ++t) {
          const bool mstep = (t == TT);
          const int i = mstep ? mid : (g ? N - 1 - t : t);
          const bool act = mstep ? (g == 0 || nb >= 1) : (t < cnt);
          const bool prev = mstep ? (cnt >= 1) : (t >= 1);
          const int cs = g ? i + 1 : i;  // the S_{cs,cs-1} this step applies
          double Sr[12];
          if (act) {
            const double* Si = DV + 78 * i;
#pragma unroll
            for (int c = 0; c < 12; ++c) Sr[c] = Si[sym_idx(pr, g ? perm12(c) : c)];
            if (prev) {
              double V[12];  // row r of D^-1 Cg^T
#pragma unroll
              for (int c = 0; c < 12; ++c) {
                double v = Dr[c] * cgk(g, cs, c, c);
                if (c < 3) v += Dr[6] * cgk(g, cs, c, 6) + Dr[7] * cgk(g, cs, c, 7) + Dr[8] * cgk(g, cs, c, 8);
                else if (c < 6) v += Dr[c + 6] * cgk(g, cs, c, c + 6);
                V[c] = v;
              }
              lds_wave_sync();
              if (own) {
#pragma unroll
                for (int c = 0; c < 12; ++c) Vs[r * 12 + c] = V[c];
              }
              lds_wave_sync();
              double X[12];  // row r of Cg V
              const double cr = cpl(cs, oRR);
#pragma unroll
              for (int c = 0; c < 12; ++c) X[c] = cr * Vs[r * 12 + c];
              if (r < 3) {
                const double c6 = cpl(cs, o6), c7 = cpl(cs, o7), c8 = cpl(cs, o8);
#pragma unroll
                for (int c = 0; c < 12; ++c) X[c] += c6 * Vs[72 + c] + c7 * Vs[84 + c] + c8 * Vs[96 + c];
              } else if (r < 6) {
                const double c9 = cpl(cs, oR6);
#pragma unroll
                for (int c = 0; c < 12; ++c) X[c] += c9 * Vs[(r + 6) * 12 + c];
              }
              if (mstep && g == 1) {
                if (own) {
#pragma unroll
                  for (int c = 0; c < 12; ++c) XB[r * 12 + c] = X[c];
                }
              } else {
#pragma unroll
                for (int c = 0; c < 12; ++c) Sr[c] -= X[c];
              }
            }
          }
          if (mstep) {
            lds_wave_sync();
            if (g == 0 && nb >= 1) {  // un-permute group 1's term: X_b[r][c] = XB[pi r][pi c]
#pragma unroll
              for (int c = 0; c < 12; ++c) Sr[c] -= XB[perm12(r) * 12 + perm12(c)];
            }
          }
          if (act && !(mstep && g == 1)) {
            inverse_rows12(Sr, Dr);
            if (own) {
              double* Di = DV + 78 * i;
#pragma unroll
              for (int c = 0; c < 12; ++c) {
                const int pc = g ? perm12(c) : c;
                if (pc <= pr) Di[pr * (pr + 1) / 2 + pc] = Dr[c];
              }
            }
          }
        }
      }
    }
    __syncthreads();
    PROF_ADD_CTX((*this), 2);
  }

  // One step of iterative refinement of a direction against the full KKT from the residuals of all
  // four rows (pdipm_srbd.hpp FastCtx::refine_rhs has the scheme, pdipm_srbd_reg.hpp RegCtx::refine_rhs
  // the derivation): step 0 per inequality row q = D^-1 (e2 - W e3), DZ += q, DS += e3 + delta q (the
  // parts of the correction of dz, ds that do not depend on the correction of dx); then
  // RX <- -(e1 - G^T q) (G^T over the updated DZ), RE <- -e4; dx and dy saved to the output rows for
  // solve(true), which adds Lambda G c_x to dz and (delta Lambda - 1) G c_x to ds. RX, RE are
  // overwritten (the caller restores them with residuals() after refining the affine direction).
  __device__ void refine_rhs() {
    for (int q = lane; q < m; q += nt) {  // step 0 (rows 2 and 3)
      const int i = q / 16, k = q % 16;
      double gd = 0.0;
      gd = grow_dot(i, k, TV + 12 * N + 12 * i, gd);
      const double e3 = -RS[q] - ((gd + DS[q]) - kDelta * DZ[q]);
      const double e2 = R2[q] - (WD[q] * DS[q] + DZ[q]);
      const double qc = DI[q] * (e2 - WD[q] * e3);
      DS[q] = DS[q] + (e3 + kDelta * qc);
      DZ[q] = DZ[q] + qc;
    }
    __syncthreads();
    for (int e = lane; e < nz; e += nt) xsg[e] = TV[e];
    for (int e = lane; e < p; e += nt) ysg[e] = DY[e];
    for (int c = lane; c < nz; c += nt) {
      double v = (HV[c] + kBeta) * TV[c] + RX[c];
      if (c >= 12 * N) {
        const int i = (c - 12 * N) / 12, j = (c - 12 * N) % 12;
        double gz = 0.0;
        gcol_dot(i, j, DZ + 16 * i, gz);
        double ay = 0.0;
        const int ub = a_ublock(N, i) + T->cpu[j];
        ay = col_dot<8>(ub, T->su_n[j], T->su[j], DY + 12 * i, ay);
        if (j == 6) ay += AV[ub + T->su_n[j]] * DY[12 * N + 2 * i];
        if (j == 9) ay += AV[ub + T->su_n[j]] * DY[12 * N + 2 * i + 1];
        v = (v + gz) + ay;
      } else {
        const int k = c / 12 + 1, j = c % 12;
        double ay;
        if (k < N) {
          const int xb = a_xblock(k) + T->cpx[j];
          ay = AV[xb] * DY[12 * (k - 1) + j];
          ay = col_dot<4>(xb + 1, T->sx_n[j], T->sx[j], DY + 12 * k, ay);
        } else {
          ay = AV[36 * (N - 1) + j] * DY[12 * (k - 1) + j];
        }
        v = v + ay;
      }
      RX[c] = v;
    }
    for (int e = lane; e < p; e += nt) {
      double v = 0.0;
      if (e < 12 * N) {
        const int i = e / 12, r = e % 12;
        if (i >= 1) v += mrow(i, r, TV + 12 * (i - 1));
        v += Pv(i, r) * TV[12 * i + r];
        v += nrow(i, r, TV + 12 * N + 12 * i);
      } else {
        const int i = (e - 12 * N) / 2, w = (e - 12 * N) % 2;
        v = (w == 0 ? E6(i) * TV[12 * N + 12 * i + 6] : E9(i) * TV[12 * N + 12 * i + 9]);
      }
      RE[e] = (v + RE[e]) - kDelta * DY[e];
    }
    __syncthreads();
    PROF_ADD_CTX((*this), 7);
  }

  // ------------------------------------------------------------------------- solve ----
  // Solves K [dx; ds; dz; dy] = [-RX; R2; -RS; -RE] with the current factors.
  // Result: dx -> TV, ds -> DS, dz -> DZ, dy -> DY.
  // ref: the refinement solve -- rhs [-RX; 0; 0; -RE] for the correction (refine_rhs's step 0 carried
  // rows 2 and 3 into DZ, DS), dx = saved + correction; DY is the correction. dz and ds move by the
  // correction's own Lambda G c_x: re-forming them from the whole dx, dz = VV + Lambda G dx, would
  // round G dx at eps |G| |dx| and multiply that by Lambda = W / (1 + delta W) -- at z / s = 6e5 it
  // left dz 1e-9 off the exact answer after the refinement (scripts/extended_precision_check.py).
  __device__ void solve(bool ref = false) {
    if (!ref)
      for (int q = lane; q < m; q += nt) VV[q] = DI[q] * (R2[q] + WD[q] * RS[q]);  // D^-1 (r2 - W r3)
    __syncthreads();
    // r1~ = r1 - G^T VV
    for (int c = lane; c < nz; c += nt) {
      double v = -RX[c];
      if (c >= 12 * N && !ref) {
        const int i = (c - 12 * N) / 12, j = (c - 12 * N) % 12;
        double g = 0.0;
        gcol_dot(i, j, VV + 16 * i, g);
        v -= g;
      }
      R1T[c] = v;
    }
    __syncthreads();
    // t = Phi^-1 r1~ (x: diagonal; u: foot blocks, scalars, x-moment pairs)
    for (int c = lane; c < 12 * N; c += nt) TV[c] = R1T[c] / phix(c / 12 + 1, c % 12);
    for (int task = lane; task < 3 * N; task += nt) {
      if (task < 2 * N) {
      const int i = task >> 1, f = task & 1;
      double rv[4], tv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) rv[a] = R1T[12 * N + 12 * i + T->foot_col[f][a]];
      ldlt_solve_p<4>(PH + 24 * i + 10 * f, rv, tv);
#pragma unroll
      for (int a = 0; a < 4; ++a) TV[12 * N + 12 * i + T->foot_col[f][a]] = tv[a];
      } else {
      const int i = task - 2 * N;
      const int b = 12 * N + 12 * i;
      const double p6 = phiu(i, 6), p9 = phiu(i, 9), e6 = E6(i), e9 = E9(i);
      const double r4a = -RE[12 * N + 2 * i], r4b = -RE[12 * N + 2 * i + 1];
      TV[b + 6] = (kDelta * R1T[b + 6] + e6 * r4a) / (p6 * kDelta + e6 * e6);
      TV[b + 9] = (kDelta * R1T[b + 9] + e9 * r4b) / (p9 * kDelta + e9 * e9);
      TV[b + 8] = R1T[b + 8] * PH[24 * i + 22];
      TV[b + 11] = R1T[b + 11] * PH[24 * i + 23];
      }
    }
    __syncthreads();
    // g = A_dyn t - r4_dyn
    for (int e = lane; e < 12 * N; e += nt) {
      const int i = e / 12, r = e % 12;
      double v = 0.0;
      if (i >= 1) v += mrow(i, r, TV + 12 * (i - 1));
      v += Pv(i, r) * TV[12 * i + r];
      v += nrow(i, r, TV + 12 * N + 12 * i);
      QV[e] = v + RE[e];
    }
    __syncthreads();
    PROF_ADD_CTX((*this), 3);
    // Twisted block solve with the factors of factor() (pdipm_srbd.hpp FastCtx::solve, per-stage couplings):
    //   elimination: group 0  q_i = g_i - C_i w_{i-1},         w_i = D_i^-1 q_i   (i = 0 .. mid-1)
    //                group 1  p_j = g_j - C_{j+1}^T v_{j+1},   v_j = E_j^-1 p_j   (j = N-1 .. mid+1)
    //   middle:      y_mid = T^-1 (g_mid - C_m w_{mid-1} - C_{m+1}^T v_{mid+1})
    //   outward:     group 0  y_i = w_i - D_i^-1 C_{i+1}^T y_{i+1};  group 1  y_j = v_j - E_j^-1 C_j y_{j-1}
    // g is read from QV, y written back to QV; w / v kept in WV. Crow / Ccol: row / column r of the
    // coupling (zeros included), DPP-broadcast products over the 16-lane group.
    {
      const int mid = N / 2, nf = mid, nb = N - 1 - mid;
      const int TT = nf > nb ? nf : nb;
      if (lane < 32) {
        const int g = lane >> 4;
        const int r = (lane & 15) < 12 ? (lane & 15) : 11;
        const bool own = (lane & 15) < 12;
        const int pr = g ? perm12(r) : r;
        const int cnt = g ? nb : nf;
        int oRow[12], oCol[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) {
          oRow[j] = cg_off(g, r, j);
          oCol[j] = cg_off(g, j, r);
        }
        double w = 0.0;
#pragma unroll 1
        for (int t = 0; t <= TT; ++t) {
          const bool mstep = (t == TT);
          const int i = mstep ? mid : (g ? N - 1 - t : t);
          const bool act = mstep ? (g == 0 || nb >= 1) : (t < cnt);
          const bool prev = mstep ? (cnt >= 1) : (t >= 1);
          double cw = 0.0;  // Cg times the previous w (both groups)
          if (act && prev) {
            const int cs = g ? i + 1 : i;
            double Crow[12];
#pragma unroll
            for (int j = 0; j < 12; ++j) Crow[j] = cg_at(cs, oRow[j]);
            double c0 = 0.0, c1 = 0.0, c2 = 0.0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              c0 += Crow[j] * bc16(w, j);
              c1 += Crow[j + 4] * bc16(w, j + 4);
              c2 += Crow[j + 8] * bc16(w, j + 8);
            }
            cw = (c0 + c1) + c2;
          }
          if (mstep) {  // group 1 hands C^T v_{mid+1} (original coordinates) to group 0
            if (g == 1 && own && nb >= 1) SC[432 + pr] = cw;
            lds_wave_sync();
          }
          if (act && !(mstep && g == 1)) {
            const double* Di = DV + 78 * i;
            double Dr[12];
#pragma unroll
            for (int k = 0; k < 12; ++k) Dr[k] = Di[sym_idx(pr, g ? perm12(k) : k)];
            double q = QV[12 * i + pr] - cw;
            if (mstep && nb >= 1) q -= SC[432 + r];
            double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              a0 += Dr[k] * bc16(q, k);
              a1 += Dr[k + 4] * bc16(q, k + 4);
              a2 += Dr[k + 8] * bc16(q, k + 8);
            }
            w = (a0 + a1) + a2;
            if (own) WV[12 * i + pr] = w;
          }
        }
        PROF_ADD_CTX((*this), 4);
        // outward substitution from the middle block (y_mid = group 0's last w, also in WV_mid)
        lds_wave_sync();
        if (own && g == 0) QV[12 * mid + r] = w;
        double y = (g == 0) ? w : WV[12 * mid + pr];
#pragma unroll 1
        for (int t = 0; t < TT; ++t) {
          const int i = g ? mid + 1 + t : mid - 1 - t;
          if (t < cnt) {
            const int cs = g ? i : i + 1;
            double Ccol[12], Dr[12];
#pragma unroll
            for (int j = 0; j < 12; ++j) Ccol[j] = cg_at(cs, oCol[j]);
            const double* Di = DV + 78 * i;
#pragma unroll
            for (int k = 0; k < 12; ++k) Dr[k] = Di[sym_idx(pr, g ? perm12(k) : k)];
            double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {  // Cg^T y_prev
              s0 += Ccol[j] * bc16(y, j);
              s1 += Ccol[j + 4] * bc16(y, j + 4);
              s2 += Ccol[j + 8] * bc16(y, j + 8);
            }
            const double sc = (s0 + s1) + s2;
            double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              a0 += Dr[k] * bc16(sc, k);
              a1 += Dr[k + 4] * bc16(sc, k + 4);
              a2 += Dr[k + 8] * bc16(sc, k + 8);
            }
            y = WV[12 * i + pr] - ((a0 + a1) + a2);
            if (own) QV[12 * i + pr] = y;
          }
        }
      }
    }
    __syncthreads();
    PROF_ADD_CTX((*this), 5);
    // dx = t - Phi^-1 A_dyn^T dy ; x-moment duals from the exact 2x2 elimination
    for (int c = lane; c < 12 * N; c += nt) {
      const int k = c / 12 + 1, j = c % 12;
      double aty;
      if (k < N) {
        const int xb = a_xblock(k) + T->cpx[j];
        aty = AV[xb] * QV[12 * (k - 1) + j];
        aty = col_dot<4>(xb + 1, T->sx_n[j], T->sx[j], QV + 12 * k, aty);
      } else {
        aty = AV[36 * (N - 1) + j] * QV[12 * (k - 1) + j];
      }
      TV[c] = ref ? xsg[c] + (TV[c] - aty / phix(k, j)) : TV[c] - aty / phix(k, j);
    }
    // (A_dyn^T dy) of every u column, one column per thread, into WV (dead after the chains): the
    // per-(stage, foot) tasks below then read them instead of each summing four columns in a row
    for (int c = lane; c < 12 * N; c += nt) {
      const int i = c / 12, j = c % 12;
      WV[c] = col_dot<8>(a_ublock(N, i) + T->cpu[j], T->su_n[j], T->su[j], QV + 12 * i, 0.0);
    }
    __syncthreads();
    for (int task = lane; task < 3 * N; task += nt) {
      // u columns: per (stage, foot) block or per stage scalars
      const bool foot = task < 2 * N;
      const int i = foot ? (task >> 1) : task - 2 * N;
      const int b = 12 * N + 12 * i;
      auto aty_u = [&](int j) { return WV[12 * i + j]; };
      if (foot) {
        const int f = task & 1;
        double av[4], tv[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) av[a] = aty_u(T->foot_col[f][a]);
        ldlt_solve_p<4>(PH + 24 * i + 10 * f, av, tv);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const int o = b + T->foot_col[f][a];
          const double cv = TV[o] - tv[a];
          if (ref) R1T[o] = cv;  // the correction of the foot columns (R1T is dead there)
          TV[o] = ref ? xsg[o] + cv : cv;
        }
      } else {
        const double p6 = phiu(i, 6), p9 = phiu(i, 9), e6 = E6(i), e9 = E9(i);
        const double r4a = -RE[12 * N + 2 * i], r4b = -RE[12 * N + 2 * i + 1];
        const double a6 = aty_u(6), a9 = aty_u(9), a8 = aty_u(8), a11 = aty_u(11);
        const double t6 = TV[b + 6] - PH[24 * i + 20] * a6, t9 = TV[b + 9] - PH[24 * i + 21] * a9;
        const double t8 = TV[b + 8] - PH[24 * i + 22] * a8, t11 = TV[b + 11] - PH[24 * i + 23] * a11;
        TV[b + 6] = ref ? xsg[b + 6] + t6 : t6;
        TV[b + 9] = ref ? xsg[b + 9] + t9 : t9;
        TV[b + 8] = ref ? xsg[b + 8] + t8 : t8;
        TV[b + 11] = ref ? xsg[b + 11] + t11 : t11;
        const double rho6 = R1T[b + 6] - a6, rho9 = R1T[b + 9] - a9;
        DY[12 * N + 2 * i] = (e6 * rho6 - p6 * r4a) / (p6 * kDelta + e6 * e6);
        DY[12 * N + 2 * i + 1] = (e9 * rho9 - p9 * r4b) / (p9 * kDelta + e9 * e9);
      }
    }
    for (int e = lane; e < 12 * N; e += nt) DY[e] = QV[e];
    __syncthreads();
    // dz = D^-1 (r2 - W r3) + Lam G dx ; ds = r3 - G dx + delta dz
    for (int q = lane; q < m; q += nt) {
      const int i = q / 16, k = q % 16;
      double gd = 0.0;
      if (ref) {  // G touches the foot columns only
        gd = grow_dot(i, k, R1T + 12 * N + 12 * i, gd);
        const double lg = DI[q] * WD[q] * gd;
        DZ[q] = DZ[q] + lg;
        DS[q] = DS[q] + (kDelta * lg - gd);
      } else {
        gd = grow_dot(i, k, TV + 12 * N + 12 * i, gd);
        const double dz = VV[q] + DI[q] * WD[q] * gd;
        DZ[q] = dz;
        DS[q] = -RS[q] - gd + kDelta * dz;
      }
    }
    __syncthreads();
    PROF_ADD_CTX((*this), 6);
  }

  // kRefineSteps refinement steps (pdipm_srbd.hpp FastCtx::refine: later steps restore the original
  // right-hand side and refine from the full dy = saved + correction)
  template <bool kInl>
  __device__ void refine() {
    for (int step = 0; step < kRefineSteps; ++step) {
      if (step > 0) {
        for (int e = lane; e < p; e += nt) DY[e] = ysg[e] + DY[e];
        SRBD_GCALL(this->residuals());
      }
      SRBD_GCALL(this->refine_rhs());
      SRBD_GCALL(this->solve(true));
    }
  }

  // fmax(fmin(1, 0.99 * min_i if_else(dv_i < 0, -v_i/dv_i, 1)), 1e-12)  (:460-467)
  __device__ double step_length(const double* v, const double* dv) const {
    double mn = INFINITY;
    for (int q = lane; q < m; q += nt) {
      const bool c = dv[q] < 0.0;
      const double a = -v[q] / dv[q];
      const double cand = (c ? a : 0.0) + (!c ? 1.0 : 0.0);
      mn = fmin(mn, cand);
    }
    mn = team_min(mn);
    return fmax(fmin(1.0, 0.99 * mn), 1e-12);
  }
};

// The general solve of QP `env` with its working set at `smem` (the workgroup's LDS in pdipm_kernel,
// a slot of the library's global scratch pool when a stage-invariant kernel meets a QP it cannot
// take). `lane_in` is the thread's index in the QP's team of `nt_in` threads: every wave of the
// workgroup (two in the general kernel; in the fallback the calling kernel's waves of that QP).
// `smem`: the QP's working set (the workgroup's LDS in pdipm_kernel, a scratch-pool slot in global
// memory for the fallback). `lds`, `lds_cap`: LDS the caller can spare (the fallback: the stage-invariant
// kernel's own LDS, unused by a QP it hands over); the arrays the sequential chains touch go there first
// -- the factor blocks, their scratch, the solve chains' vectors -- then the row-parallel ones, as long
// as they fit; the rest stay in `smem`. (Global-memory latency on every chain step is what made the
// fallback ~2x slower than the same solve in LDS.)
template <bool kInl>
__device__ __forceinline__ void pdipm_general_at(const SolverArgs& args, int env, double* smem, int lane_in,
                                                 int nt_in, int status_bits = 0, double* lds = nullptr,
                                                 int lds_cap = 0) {
  const int N = args.N;
  const SolverLayout Lo(N);
  SolverCtx C;
  C.N = N;
  C.nz = 24 * N;
  C.m = 16 * N;
  C.p = 14 * N;
  C.nd = 12 * N;
  C.lane = lane_in;
  C.nt = nt_in;
  {
    int used = 0;
    auto place = [&](double*& ptr, int off, int n) {
      const int n2 = (n + 1) & ~1;
      if (lds && used + n2 <= lds_cap) {
        ptr = lds + used;
        used += n2;
      } else {
        ptr = smem + off;
      }
    };
    const int nz = C.nz, m = C.m, p = C.p, nd = C.nd;
    double* tb = nullptr;
    place(tb, Lo.TB, kTablesDoubles);
    const bool tb_lds = lds == nullptr || tb != smem + Lo.TB;  // an LDS copy (else read c_tab itself)
    C.T = tb_lds ? reinterpret_cast<const Tables*>(tb) : &c_tab;
    if (tb_lds) {  // copy the tables, 2 bytes per lane and pass (Tables is 2-byte aligned)
      static_assert(sizeof(Tables) % 2 == 0 && alignof(Tables) <= 16, "Tables copy");
      const uint16_t* src = reinterpret_cast<const uint16_t*>(&c_tab);
      uint16_t* dst = reinterpret_cast<uint16_t*>(tb);
      for (int w = lane_in; w < (int)(sizeof(Tables) / 2); w += C.nt) dst[w] = src[w];
    }
    if (Lo.CV >= 0) place(C.CV, Lo.CV, 36 * N);
    else C.CV = nullptr;
    C.KX = nullptr;
    if constexpr (kInl)
      if (Lo.KX >= 0) place(C.KX, Lo.KX, 78 * N);
    place(C.DV, Lo.DV, 78 * N); place(C.SC, Lo.SC, 448); place(C.RD, Lo.RD, 8); place(C.QV, Lo.QV, nd); place(C.WV, Lo.WV, nd);
    place(C.PH, Lo.PH, 24 * N); place(C.TV, Lo.TV, nz); place(C.R1T, Lo.R1T, nz);
    place(C.DI, Lo.DI, m); place(C.WD, Lo.WD, m); place(C.SI, Lo.SI, m); place(C.VV, Lo.VV, m);
    place(C.R2, Lo.R2, m); place(C.DS, Lo.DS, m); place(C.DZ, Lo.DZ, m); place(C.DY, Lo.DY, p);
    place(C.X, Lo.X, nz); place(C.S, Lo.S, m); place(C.Z, Lo.Z, m); place(C.Y, Lo.Y, p);
    place(C.RX, Lo.RX, nz); place(C.RS, Lo.RS, m); place(C.RE, Lo.RE, p);
    place(C.HV, Lo.HV, nz); place(C.GV, Lo.GV, 28 * N); place(C.AV, Lo.AV, 122 * N - 24);
  }
  const int lane = C.lane, nz = C.nz, m = C.m, p = C.p, nt = C.nt;
  const int nA = nnz_A(N), nG = 28 * N;
  const double* Hg = solver_in(args, 0) + (size_t)env * nz;
  const double* Gg = solver_in(args, 1) + (size_t)env * nG;
  const double* Ag = solver_in(args, 2) + (size_t)env * nA;
  C.fg = solver_in(args, 3) + (size_t)env * nz;
  C.hg = solver_in(args, 4) + (size_t)env * m;
  C.bg = solver_in(args, 5) + (size_t)env * p;
  C.xsg = solver_out(args, 0) + (size_t)env * nz;
  C.ysg = solver_out(args, 3) + (size_t)env * p;
  for (int e = lane; e < nA; e += nt) C.AV[e] = Ag[e];
  for (int e = lane; e < nG; e += nt) C.GV[e] = Gg[e];
  for (int e = lane; e < nz; e += nt) C.HV[e] = Hg[e];
  if (args.init_mode == 2) {  // _ccs cold start (sparse_pdipm_solver.py:30-35)
    const double* xg = solver_in(args, 6) + (size_t)env * nz;
    for (int e = lane; e < nz; e += nt) C.X[e] = xg[e];
    __syncthreads();
    for (int e = lane; e < m; e += nt) { C.S[e] = fmax(C.hg[e] - ccs_gx(Gg, e, C.X + 12 * N), 1.0); C.Z[e] = 1.0; }
    for (int e = lane; e < p; e += nt) C.Y[e] = 0.0;
  } else if (args.init_mode == 0) {
    const double* xg = solver_in(args, 6) + (size_t)env * nz;
    const double* sg = solver_in(args, 7) + (size_t)env * m;
    const double* zg = solver_in(args, 8) + (size_t)env * m;
    const double* yg = solver_in(args, 9) + (size_t)env * p;
    for (int e = lane; e < nz; e += nt) C.X[e] = xg[e];
    for (int e = lane; e < m; e += nt) { C.S[e] = sg[e]; C.Z[e] = zg[e]; }
    for (int e = lane; e < p; e += nt) C.Y[e] = yg[e];
  } else {
    // mpc_controller_cusadi.py:138-141: x = 0, s = max(d - G 0, 1), z = 1, y = y0
    for (int e = lane; e < nz; e += nt) C.X[e] = 0.0;
    for (int e = lane; e < m; e += nt) { C.S[e] = fmax(C.hg[e] - 0.0, 1.0); C.Z[e] = 1.0; }
    for (int e = lane; e < p; e += nt) C.Y[e] = args.y0;
  }
  __syncthreads();
  C.template couplings<kInl>();
  __syncthreads();

  double res0 = 0.0, res1 = 0.0, res2 = 0.0, mu_new = 0.0;
  bool floor_hit = false;
  PROF_MARK_CTX(C);
  for (int it = 0; it < args.n_iter; ++it) {
    double mu;
    SRBD_GCALL(mu = C.residuals());
    PROF_ADD_CTX(C, 0);
    if (it == args.n_iter - 1) {  // residual norms of the last iteration (refine_rhs reuses RX, RE)
      double a = 0.0, b = 0.0, c = 0.0;
      for (int e = lane; e < nz; e += nt) a += C.RX[e] * C.RX[e];
      for (int e = lane; e < m; e += nt) b += C.RS[e] * C.RS[e];
      for (int e = lane; e < p; e += nt) c += C.RE[e] * C.RE[e];
      res0 = sqrt(C.team_sum(a));
      res1 = sqrt(C.team_sum(b));
      res2 = sqrt(C.team_sum(c));
    }
    SRBD_GCALL(C.factor());
    // affine: r2 = -(S^-1 (s o z))
    for (int q = lane; q < m; q += nt) C.R2[q] = -(C.SI[q] * (C.S[q] * C.Z[q]));
    __syncthreads();
    SRBD_GCALL(C.solve());
    SRBD_GCALL(C.template refine<kInl>());  // the affine direction too (pdipm_srbd.hpp main loop: its ds, dz feed sigma)
    SRBD_GCALL(C.residuals());  // restores RX, RS, RE for the combined solve
    PROF_ADD_CTX(C, 0);
    double ap, ad;
    SRBD_GCALL(ap = C.step_length(C.S, C.DS));
    SRBD_GCALL(ad = C.step_length(C.Z, C.DZ));
    double sza = 0.0;
    for (int q = lane; q < m; q += nt) sza += (C.S[q] + ap * C.DS[q]) * (C.Z[q] + ad * C.DZ[q]);
    const double mu_aff = C.team_sum(sza) / m;
    const double sigma = pow(mu_aff / mu, 3.0);
    // combined rhs: r2 = -(S^-1 (s o z)) - S^-1 (s o z + ds_a o dz_a - sigma mu e)
    __syncthreads();
    for (int q = lane; q < m; q += nt) {
      const double rc = C.S[q] * C.Z[q] + C.DS[q] * C.DZ[q] - sigma * mu * 1.0;
      C.R2[q] = -(C.SI[q] * (C.S[q] * C.Z[q])) + -(C.SI[q] * rc);
    }
    __syncthreads();
    SRBD_GCALL(C.solve());
    SRBD_GCALL(C.template refine<kInl>());
    double apc, adc;
    SRBD_GCALL(apc = C.step_length(C.S, C.DS));
    SRBD_GCALL(adc = C.step_length(C.Z, C.DZ));
    floor_hit = apc <= 1e-12 || adc <= 1e-12;  // the last iteration's value is reported
    __syncthreads();
    double szn = 0.0;
    for (int e = lane; e < nz; e += nt) C.X[e] = C.X[e] + apc * C.TV[e];
    for (int q = lane; q < m; q += nt) {
      const double sn = fmax(C.S[q] + apc * C.DS[q], 1e-8);
      const double zn = fmax(fmax(C.Z[q] + adc * C.DZ[q], 1e-8), 1e-8);
      C.S[q] = sn;
      C.Z[q] = zn;
      szn += sn * zn;
    }
    for (int e = lane; e < p; e += nt) C.Y[e] = C.Y[e] + adc * (C.ysg[e] + C.DY[e]);  // saved + correction
    mu_new = C.team_sum(szn) / m;
    __syncthreads();
    PROF_ADD_CTX(C, 8);
  }
  PROF_FLUSH(C);
  double* xo = solver_out(args, 0) + (size_t)env * nz;
  double* so = solver_out(args, 1) + (size_t)env * m;
  double* zo = solver_out(args, 2) + (size_t)env * m;
  double* yo = solver_out(args, 3) + (size_t)env * p;
  double* ro = solver_out(args, 4) + (size_t)env * 4;
  double* mo = solver_out(args, 5) + (size_t)env;
  for (int e = lane; e < nz; e += nt) xo[e] = C.X[e];
  for (int e = lane; e < m; e += nt) { so[e] = C.S[e]; zo[e] = C.Z[e]; }
  for (int e = lane; e < p; e += nt) yo[e] = C.Y[e];
  if (lane == 0) {
    ro[0] = res0;
    ro[1] = res1;
    ro[2] = res2;
    ro[3] = mu_new;
    mo[0] = mu_new;
  }
  if (args.status) {
    bool nf = lane == 0 && not_finite(mu_new);
    for (int e = lane; e < nz; e += nt) nf = nf || not_finite(C.X[e]);
    for (int e = lane; e < m; e += nt) nf = nf || not_finite(C.S[e]) || not_finite(C.Z[e]);
    for (int e = lane; e < p; e += nt) nf = nf || not_finite(C.Y[e]);
    nf = C.team_sum(nf ? 1.0 : 0.0) > 0.0;
    if (lane == 0)
      args.status[env] = status_bits | (nf ? kStatusNonFinite : 0) | (floor_hit ? kStatusStepFloor : 0);
  }
}

// A QP the stage-invariant kernels cannot take (not stage-invariant: any CCS input other than
// qp_former's output), solved inside the same launch by the workgroup that found it, in a slot of
// the library's scratch pool (global memory, L2-resident): lane 0 takes a free slot by its lock word
// (a slot holder is a running workgroup that releases it when done, so the spin ends), the solve runs
// with the slot as its working set, and the slot's writes are released (agent-scope fence) before its
// lock. Not inlined: the stage-invariant kernels keep their own register allocation; one copy per
// calling kernel (kTag), so each is compiled under its caller's occupancy target (the register
// kernels' 2 waves per SIMD). A qp_former batch never gets here, so the fast path pays nothing for
// it (no second launch, no flag pass).
// `args` is the kernel's own argument, addressed in the kernarg segment (kernel_args()): taking the
// address of the by-value kernel parameter instead would copy it to scratch and make the caller
// read every argument from there.
__device__ __forceinline__ const SolverArgs& kernel_args() {
  return *(const SolverArgs*)__builtin_amdgcn_kernarg_segment_ptr();  // constant -> generic address space
}
// `lds` / `lds_doubles`: the calling workgroup's LDS (all of it: the QP handed over never started the
// fast path); its first int is where a multi-wave QP's waves agree on the slot (wave 0 takes it; all
// of the QP's waves then run the solve as one team over the slot's memory),
// the rest holds the chain arrays of the general solve (pdipm_general_at). The pool has as many slots
// as the device holds resident workgroups of any stage-invariant kernel, so a slot is free at the first
// or an early probe and no workgroup waits on another's solve.
template <int kTag>
__device__ __attribute__((noinline)) void pdipm_general_scratch(const SolverArgs& args, int env, double* lds,
                                                                int lds_doubles) {
  const int n = args.scratch_slots;
  int slot = env % n;
  int* xchg = reinterpret_cast<int*>(lds);
  if (threadIdx.x == 0) {
    while (atomicCAS(&args.scratch_locks[(size_t)slot * kLockStride], 0, 1) != 0) {
      slot = slot + 1 == n ? 0 : slot + 1;
      __builtin_amdgcn_s_sleep(8);
    }
    *xchg = slot;
  }
  __syncthreads();
  slot = *xchg;
  __syncthreads();  // every wave has the slot before the general solve reuses the LDS
  __threadfence();
  pdipm_general_at<false>(args, env, args.scratch + (size_t)slot * args.scratch_stride, threadIdx.x,
                          blockDim.x, kStatusFallback, lds, lds_doubles);
  __syncthreads();
  __threadfence();
  if (threadIdx.x == 0) atomicExch(&args.scratch_locks[(size_t)slot * kLockStride], 0);
}

#ifndef SRBD_NO_GENERAL_KERNEL  // srbd_reg20.hip (second unit) does not define it again
// One workgroup per QP (the "general" solver path, srbd_set_solver_path(1))
__global__ __launch_bounds__(kGeneralThreads) void pdipm_kernel(SolverArgs args) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  if ((int)blockIdx.x < args.batch) pdipm_general_at<true>(args, blockIdx.x, smem, threadIdx.x, kGeneralThreads);
}
#endif  // SRBD_NO_GENERAL_KERNEL

}  // namespace srbd
