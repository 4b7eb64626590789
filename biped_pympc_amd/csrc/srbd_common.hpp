// srbd_common.hpp -- shared definitions for the SRBD-MPC HIP kernels (gfx950 / CDNA4, wave64).
//
// Stage-periodic sparsity tables of the QP produced by qp_former (reference
// biped_pympc/casadi/srbd_constraints.py:83-227; CCS convention sparse_pdipm_solver.py:561-591).
// The same closed-form rules live in biped_pympc_amd/layout.py; tests/test_layout.py checks that
// both agree with a structural dependency analysis of the literal RK4 model.
//
// Decision vector z = [x_1..x_N, u_0..u_{N-1}];  x_k[j] -> 12(k-1)+j,  u_i[j] -> 12N+12i+j.
// Rows: dynamics of stage i -> 12i+r ; x-moment rows -> 12N+2i+{0,1} ; inequalities -> 16i+8f+k.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace srbd {

constexpr double kBeta = 1e-8;    // generate_solver_function.py:112
constexpr double kDelta = 1e-8;   // sparse_pdipm_solver.py:416
constexpr double kFMax = 500.0;   // srbd_constraints.py:31
constexpr double kLt = 0.07;      // srbd_constraints.py:161
constexpr double kLh = 0.04;      // srbd_constraints.py:162
constexpr double kGravZ = -9.81;  // srbd_centroidal_model.py:136
constexpr int kMaxN = 32;         // horizon supported by the kernels (LDS-bound)

struct Tables {
  // S_x(j): stage-local rows touched by x_i[j] through -A_d (count sx_n[j], rows sx[j][t]).
  int8_t sx_n[12];
  int8_t sx[12][4];
  // S_u(j): stage-local rows touched by u_i[j] through -B_d.
  int8_t su_n[12];
  int8_t su[12][8];
  // CCS column offsets inside one periodic block (x block = 36 values, u block = 86 values).
  int16_t cpx[12];  // start of column x_k[j] inside the 36-value block of x_k (k < N)
  int16_t cpu[12];  // start of column u_i[j] inside the 86-value block of u_i
  int16_t e6, e9;   // x-moment entries (rows 12N+2i, 12N+2i+1) inside the u_i block
  // Dense 12x12 stage-local index maps into the periodic blocks (-1 = structural zero):
  //   Mi[r][j]: entry of M_i = (stage i rows, x_i columns)  -> offset inside x_i's 36-block
  //   Ni[r][j]: entry of N_i = (stage i rows, u_i columns)  -> offset inside u_i's 86-block
  int16_t Mi[12][12];
  int16_t Ni[12][12];
  // G: 28 values per stage in CCS order; gcol/grow give the (u column, stage-local row) pair.
  int8_t gcol[28];
  int8_t grow[28];
  // Row-wise view of G: row k (0..15) -> up to 2 entries (value offset, u column).
  int8_t gr_n[16];
  int8_t gr_off[16][2];
  int8_t gr_col[16][2];
  // Inverse of cpx/cpu: (row, column) of each offset inside one x block (36) / u block (86);
  // row -1 = the +I entry of an x column, row 12/13 = the x-moment entries e6/e9 of a u block.
  int8_t xb_r[36], xb_j[36];
  int8_t ub_r[86], ub_j[86];
  // Packed-lower 12x12 entries (row | col << 4, row >= col) in the lane order of the S_ii build:
  // rows/cols {0,1,2,6,7,8} meet every foot column of N ("dense"), rows {3,4,5,9,10,11} exactly one
  // per foot (position r % 3). 21 dense-dense entries, then the 57 with a sparse index; within each
  // class the order minimises the bank conflicts of the entries' LDS stores (kSiiOrder).
  uint8_t dvo[78];
  // Foot blocks of Phi_u: u columns {0,1,2,7} (left) and {3,4,5,10} (right).
  int8_t foot_col[2][4];
  // column -> (foot, position) or -1 for the four decoupled columns {6,8,9,11}
  int8_t col_foot[12];
  int8_t col_pos[12];
  // G by column: u column j's entries are gcp[j] .. gcp[j] + gcn[j] - 1 in CCS order (at most 8)
  int8_t gcp[12], gcn[12];
};

// kSiiOrder: scripts/sii_order.py (a seeded search over the order within each class: the extra
// LDS cycles of a stage block's ds_write_b64 fall from 6 to 5 (dense pass) and 4 to 1 (sparse pass)
// per instruction against the class-sorted row-major order; tests/test_layout.py checks the classes)
constexpr uint8_t kSiiOrder[78] = {120, 0,   23,  38,  24,  103, 17,  136, 104, 7,   102, 18,  40,  119, 22,  1,
                                   34,  2,   8,   6,   39,  20,  58,  68,  86,  85,  35,  37,  91,  56,  71,  88,
                                   121, 9,   107, 25,  3,   57,  75,  52,  139, 69,  154, 106, 170, 51,  171, 73,
                                   11,  55,  72,  123, 187, 53,  74,  137, 36,  10,  41,  70,  89,  21,  155, 105,
                                   54,  27,  59,  90,  43,  87,  26,  153, 4,   19,  42,  5,   138, 122};

constexpr Tables make_tables() {
  Tables t{};
  for (int j = 0; j < 12; ++j) {
    if (j <= 5) {
      t.sx_n[j] = 1;
      t.sx[j][0] = (int8_t)j;
    } else if (j <= 8) {
      t.sx_n[j] = 4;
      t.sx[j][0] = 0; t.sx[j][1] = 1; t.sx[j][2] = 2; t.sx[j][3] = (int8_t)j;
    } else {
      t.sx_n[j] = 2;
      t.sx[j][0] = (int8_t)(j - 6); t.sx[j][1] = (int8_t)j;
    }
    if (j <= 2) {
      const int8_t r[8] = {0, 1, 2, (int8_t)(3 + j), 6, 7, 8, (int8_t)(9 + j)};
      t.su_n[j] = 8;
      for (int q = 0; q < 8; ++q) t.su[j][q] = r[q];
    } else if (j <= 5) {
      const int8_t r[8] = {0, 1, 2, (int8_t)j, 6, 7, 8, (int8_t)(6 + j)};
      t.su_n[j] = 8;
      for (int q = 0; q < 8; ++q) t.su[j][q] = r[q];
    } else {
      const int8_t r[6] = {0, 1, 2, 6, 7, 8};
      t.su_n[j] = 6;
      for (int q = 0; q < 6; ++q) t.su[j][q] = r[q];
    }
  }
  int acc = 0;
  for (int j = 0; j < 12; ++j) {
    t.cpx[j] = (int16_t)acc;
    acc += 1 + t.sx_n[j];
  }
  acc = 0;
  for (int j = 0; j < 12; ++j) {
    t.cpu[j] = (int16_t)acc;
    acc += t.su_n[j] + ((j == 6 || j == 9) ? 1 : 0);
  }
  t.e6 = (int16_t)(t.cpu[6] + t.su_n[6]);
  t.e9 = (int16_t)(t.cpu[9] + t.su_n[9]);
  for (int j = 0; j < 12; ++j) {
    t.xb_r[t.cpx[j]] = -1;
    t.xb_j[t.cpx[j]] = (int8_t)j;
    for (int q = 0; q < t.sx_n[j]; ++q) {
      t.xb_r[t.cpx[j] + 1 + q] = t.sx[j][q];
      t.xb_j[t.cpx[j] + 1 + q] = (int8_t)j;
    }
    for (int q = 0; q < t.su_n[j]; ++q) {
      t.ub_r[t.cpu[j] + q] = t.su[j][q];
      t.ub_j[t.cpu[j] + q] = (int8_t)j;
    }
    if (j == 6 || j == 9) {
      t.ub_r[t.cpu[j] + t.su_n[j]] = (int8_t)(j == 6 ? 12 : 13);
      t.ub_j[t.cpu[j] + t.su_n[j]] = (int8_t)j;
    }
  }
  for (int r = 0; r < 12; ++r)
    for (int j = 0; j < 12; ++j) {
      t.Mi[r][j] = -1;
      t.Ni[r][j] = -1;
    }
  for (int j = 0; j < 12; ++j) {
    for (int q = 0; q < t.sx_n[j]; ++q) t.Mi[t.sx[j][q]][j] = (int16_t)(t.cpx[j] + 1 + q);
    for (int q = 0; q < t.su_n[j]; ++q) t.Ni[t.su[j][q]][j] = (int16_t)(t.cpu[j] + q);
  }
  // G per stage (srbd_constraints.py:193-222), CCS order over u columns 0..11
  int g = 0;
  for (int j = 0; j < 12; ++j) {
    int rows[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int n = 0;
    const int f = (j == 3 || j == 4 || j == 5 || j == 10) ? 1 : 0;
    const int o = 8 * f;
    if (j == 0 || j == 3) { rows[0] = o + 0; rows[1] = o + 1; n = 2; }
    if (j == 1 || j == 4) { rows[0] = o + 2; rows[1] = o + 3; n = 2; }
    if (j == 2 || j == 5) { for (int q = 0; q < 8; ++q) rows[q] = o + q; n = 8; }
    if (j == 7 || j == 10) { rows[0] = o + 4; rows[1] = o + 5; n = 2; }
    for (int q = 0; q < n; ++q) {
      t.gcol[g] = (int8_t)j;
      t.grow[g] = (int8_t)rows[q];
      ++g;
    }
  }
  for (int j = 0; j < 12; ++j) {
    t.gcn[j] = 0;
    t.gcp[j] = -1;
  }
  for (int q = 0; q < 28; ++q) {
    if (t.gcp[t.gcol[q]] < 0) t.gcp[t.gcol[q]] = (int8_t)q;
    t.gcn[t.gcol[q]]++;
  }
  for (int j = 0; j < 12; ++j)
    if (t.gcp[j] < 0) t.gcp[j] = 0;
  for (int k = 0; k < 16; ++k) t.gr_n[k] = 0;
  for (int q = 0; q < 28; ++q) {
    const int k = t.grow[q];
    t.gr_off[k][t.gr_n[k]] = (int8_t)q;
    t.gr_col[k][t.gr_n[k]] = t.gcol[q];
    t.gr_n[k]++;
  }
  for (int o = 0; o < 78; ++o) t.dvo[o] = kSiiOrder[o];
  const int8_t fl[4] = {0, 1, 2, 7}, fr[4] = {3, 4, 5, 10};
  for (int q = 0; q < 4; ++q) {
    t.foot_col[0][q] = fl[q];
    t.foot_col[1][q] = fr[q];
  }
  for (int j = 0; j < 12; ++j) {
    t.col_foot[j] = -1;
    t.col_pos[j] = -1;
  }
  for (int f = 0; f < 2; ++f)
    for (int q = 0; q < 4; ++q) {
      t.col_foot[t.foot_col[f][q]] = (int8_t)f;
      t.col_pos[t.foot_col[f][q]] = (int8_t)q;
    }
  return t;
}

// XCD-aware block -> work-item map. Workgroups are dealt round-robin over the 8 XCDs (block b on
// XCD b % 8; MI355X_MICROARCH.md, workgroup dispatch), and each XCD has its own L2: give XCD x one
// CONTIGUOUS range of items, so the 128-byte lines of the small per-env input rows (dt, m, mu,
// R_body, feet, ... 8-96 B each) are fetched by one L2 instead of up to eight. Placement is a speed
// hint only: the map is a bijection on [0, G), so results never depend on it.
__host__ __device__ constexpr int xcd_item(int b, int G) {
  const int x = b & 7, q = G >> 3, r = G & 7;
  return x * q + (x < r ? x : r) + (b >> 3);
}
constexpr bool xcd_item_is_bijection(int G) {  // every item hit exactly once
  unsigned long long seen[8] = {};
  for (int b = 0; b < G; ++b) {
    const int e = xcd_item(b, G);
    if (e < 0 || e >= G || (seen[e >> 6] >> (e & 63) & 1)) return false;
    seen[e >> 6] |= 1ull << (e & 63);
  }
  return true;
}
static_assert(xcd_item_is_bijection(1) && xcd_item_is_bijection(7) && xcd_item_is_bijection(8) &&
                  xcd_item_is_bijection(13) && xcd_item_is_bijection(64) && xcd_item_is_bijection(509),
              "xcd_item must permute [0, G)");

// Pattern tables in constant memory (one translation unit: srbd_mpc.hip).
static __constant__ Tables c_tab = make_tables();

// Value offsets inside A_val for horizon N.
__host__ __device__ inline int a_xblock(int k) { return 36 * (k - 1); }  // x_k block, k < N
__host__ __device__ inline int a_ubase(int N) { return 36 * N - 24; }
__host__ __device__ inline int a_ublock(int N, int i) { return 36 * N - 24 + 86 * i; }
__host__ __device__ inline int nnz_A(int N) { return 122 * N - 24; }

// Offset in A_val of the +I entry of x_{i+1}[r] (stage i rows): a full x-column block for
// i < N-1, the single-entry x_N column for the last stage.
__host__ __device__ inline int a_pidx(const Tables& t, int N, int i, int r) {
  return (i < N - 1) ? a_xblock(i + 1) + t.cpx[r] : 36 * (N - 1) + r;
}

// ------------------------------------------------------------------ phase markers ----
// Phase boundaries of the solver kernels, empty in the product build. The diagnostic builds of
// scripts/phase_profile.py / isa_phase_mix.py / prologue_profile.py force-include
// scripts/phase_prof.hpp (hipcc -include), which defines them first as s_memtime stamps.
#ifndef PROF_DECL
#define PROF_MARK_CTX(ctx)
#define PROF_ADD_CTX(ctx, k)
#define PROF_DECL
#define PROF_MARK()
#define PROF_ADD(k)
#define PROF_FLUSH(ctx)
#define PROF_SPAN(k, t0)  // cycles since t0 into slot k (t0 from PROF_NOW)
#define PROF_NOW() 0ull
#endif

// 1/d: v_rcp_f64 (~2^-24 relative) refined by the cubic step y (1 + e + e^2), e = 1 - d y: correctly
// rounded on 4M log-uniform samples (scripts/microbench_fp64.hip), i.e. the reference's IEEE 1 / d, for
// three dependent FMAs. Round 6: the Newton step y (1 + e) alone (~2^-46 relative, -DSRBD_RCP_NEWTON),
// the product's choice since round 1 (profiles/r01/rcp_variants.txt: -0.6 % at N = 10, parity magnitudes
// in the tests unchanged), left the parity campaign's register kernels at 7 / 11 failing cases of 6657
// per sequence where correctly rounded reciprocals give 3 / 2 -- through the solves' pivots (the 12x12
// chain blocks, the 4x4 foot blocks): correctly rounded W = z / s, 1 / s and step-length ratios alone left
// the counts unchanged (profiles/r06/rcp_*/).
#ifndef SRBD_RCP_NEWTON
#define SRBD_RCP_NEWTON 0
#endif
__device__ __forceinline__ double rcp3(double d) {
  const double y = __builtin_amdgcn_rcp(d);
  const double e = fma(-d, y, 1.0);
  if constexpr (SRBD_RCP_NEWTON) return fma(y, e, y);
  return fma(y, fma(e, e, e), y);
}

// ------------------------------------------------------------------ wave64 reductions ----
// DPP tree in the VALU (no LDS round trips): quads, half-rows, rows through quad_perm / mirrors,
// then row_bcast:15 / row_bcast:31 fold the four 16-lane rows into lane 63, read back uniformly.
// Rows left out by a row_mask see `id`, the operation's identity. All 64 lanes must be active.
// The first four levels read a valid lane everywhere, so they are plain DPP moves (no old value to
// materialise first: two v_mov_b32 fewer per level).
template <class Op>
__device__ __forceinline__ double wave_reduce(double v, double id, Op op) {
  v = op(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
  v = op(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true));   // quad_perm [2,3,0,1]
  v = op(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, true));  // row_half_mirror
  v = op(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xF, 0xF, true));  // row_mirror
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xA, 0xF, false));  // row_bcast:15 -> rows 1, 3
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xC, 0xF, false));  // row_bcast:31 -> rows 2, 3
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// Two independent reductions as one interleaved tree: each level's DPP moves and ops of the two
// values are independent, so the second hides the first's DPP -> VALU latency (same results as two
// wave_reduce calls, level by level).
template <class Op>
__device__ __forceinline__ void wave_reduce2(double& a, double& b, double id, Op op) {
  a = op(a, __builtin_amdgcn_mov_dpp(a, 0xB1, 0xF, 0xF, true));
  b = op(b, __builtin_amdgcn_mov_dpp(b, 0xB1, 0xF, 0xF, true));
  a = op(a, __builtin_amdgcn_mov_dpp(a, 0x4E, 0xF, 0xF, true));
  b = op(b, __builtin_amdgcn_mov_dpp(b, 0x4E, 0xF, 0xF, true));
  a = op(a, __builtin_amdgcn_mov_dpp(a, 0x141, 0xF, 0xF, true));
  b = op(b, __builtin_amdgcn_mov_dpp(b, 0x141, 0xF, 0xF, true));
  a = op(a, __builtin_amdgcn_mov_dpp(a, 0x140, 0xF, 0xF, true));
  b = op(b, __builtin_amdgcn_mov_dpp(b, 0x140, 0xF, 0xF, true));
  a = op(a, __builtin_amdgcn_update_dpp(id, a, 0x142, 0xA, 0xF, false));
  b = op(b, __builtin_amdgcn_update_dpp(id, b, 0x142, 0xA, 0xF, false));
  a = op(a, __builtin_amdgcn_update_dpp(id, a, 0x143, 0xC, 0xF, false));
  b = op(b, __builtin_amdgcn_update_dpp(id, b, 0x143, 0xC, 0xF, false));
  const long long ba = __double_as_longlong(a), bb = __double_as_longlong(b);
  const int alo = __builtin_amdgcn_readlane((int)ba, 63), ahi = __builtin_amdgcn_readlane((int)(ba >> 32), 63);
  const int blo = __builtin_amdgcn_readlane((int)bb, 63), bhi = __builtin_amdgcn_readlane((int)(bb >> 32), 63);
  a = __longlong_as_double(((long long)ahi << 32) | (unsigned int)alo);
  b = __longlong_as_double(((long long)bhi << 32) | (unsigned int)blo);
}
__device__ inline void wave_min2(double& a, double& b) {
  wave_reduce2(a, b, INFINITY, [](double x, double y) { return fmin(x, y); });
}
__device__ inline double wave_sum(double v) {
  return wave_reduce(v, 0.0, [](double a, double b) { return a + b; });
}
__device__ inline double wave_min(double v) {
  return wave_reduce(v, INFINITY, [](double a, double b) { return fmin(a, b); });
}

}  // namespace srbd
