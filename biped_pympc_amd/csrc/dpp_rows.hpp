// dpp_rows.hpp -- register-resident row primitives on 16-lane DPP rows (gfx950): broadcasts, the
// fused broadcast-FMA, and the Gauss-Jordan inverse of a 12x12 block held one row per lane. Shared by
// the LDS-resident stage-invariant kernels (pdipm_srbd.hpp), the register kernels
// (pdipm_srbd_reg.hpp) and the twisted chains of the general solve (pdipm.hpp).
#pragma once
#include "srbd_common.hpp"

namespace srbd {

// lane k of every 16-lane DPP row -> the whole row (k compile-time after unrolling); one
// v_mov_b64_dpp row_newbcast (gfx90a+ 64-bit DPP) per broadcast
#define SRBD_BC16_CASE(K) \
  case K:                 \
    return __builtin_amdgcn_mov_dpp(v, 0x150 + K, 0xF, 0xF, true);
__device__ __forceinline__ double bc16(double v, int k) {
  switch (k) {
    SRBD_BC16_CASE(0) SRBD_BC16_CASE(1) SRBD_BC16_CASE(2) SRBD_BC16_CASE(3)
    SRBD_BC16_CASE(4) SRBD_BC16_CASE(5) SRBD_BC16_CASE(6) SRBD_BC16_CASE(7)
    SRBD_BC16_CASE(8) SRBD_BC16_CASE(9) SRBD_BC16_CASE(10) SRBD_BC16_CASE(11)
    default: return v;
  }
}

// LDS hand-off between lanes of ONE wavefront: DS ops of a wave complete in order, so only the
// compiler must be kept from reordering; the wait also drains outstanding LDS ops.
__device__ __forceinline__ void lds_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// (j + 6) mod 12: swaps the (euler, position) and (omega, velocity) halves of the SRBD state
__host__ __device__ constexpr int perm12(int j) { return j < 6 ? j + 6 : j - 6; }

// ---- fused broadcast-FMA: v_fmac_f64_dpp row_newbcast:K (gfx90a+ 64-bit DPP on a VOP2 FMA) ----
// acc += v[lane K of this 16-lane row] * c in one instruction (measured 8-9 issue cycles vs ~11 for
// v_mov_b64_dpp + v_fmac_f64; scripts/microbench_fp64.hip). LLVM does not form these itself, so
// they are inline asm; an asm block is invisible to the hazard recognizer, hence the s_nop 1 on
// entry (VALU write -> DPP read needs 2 wait states, for EVERY VGPR the DPP reads, its fmac
// accumulator included). Inside a block a DPP reads no register written by one of the 2
// instructions before it (independent accumulators, or an s_nop 0 between).
// No wait states at the END of a block: the safeguard for a DPP the compiler emits after a block is
// the static audit of the final ISA (tests/test_isa_hazards.py, scripts/dpp_hazard_check.py: every
// DPP operand, every control-flow predecessor), not the hazard recognizer, which does not model
// inline asm. Dropping the trailing s_nop 1 of every block (231 per N=10 step kernel) was
// bit-identical and 1.5 % (N = 10) / 2.0 % (N = 20) faster; -DSRBD_ASM_TAIL='"s_nop 1\n"' restores
// it (A/B switch).
#ifndef SRBD_ASM_TAIL
#define SRBD_ASM_TAIL ""
#endif
#define SRBD_FMAC_BC(D, S, C, K) "v_fmac_f64_dpp " D ", " S ", " C " row_newbcast:" #K " row_mask:0xf bank_mask:0xf\n"

// one Gauss-Jordan pivot update: S[j] -= S[j](lane K) * t for the 11 columns j != K (the caller
// overwrites S[K]); row_newbcast needs K at compile time, hence one asm block per K
#define SRBD_FMAC11(K)                                                                              \
  SRBD_FMAC_BC("%0", "%0", "-%11", K) SRBD_FMAC_BC("%1", "%1", "-%11", K) SRBD_FMAC_BC("%2", "%2", "-%11", K) \
  SRBD_FMAC_BC("%3", "%3", "-%11", K) SRBD_FMAC_BC("%4", "%4", "-%11", K) SRBD_FMAC_BC("%5", "%5", "-%11", K) \
  SRBD_FMAC_BC("%6", "%6", "-%11", K) SRBD_FMAC_BC("%7", "%7", "-%11", K) SRBD_FMAC_BC("%8", "%8", "-%11", K) \
  SRBD_FMAC_BC("%9", "%9", "-%11", K) SRBD_FMAC_BC("%10", "%10", "-%11", K)
#define SRBD_PIVOT11(K, a, b, c, d, e, f, g, h, i, j, l)                                             \
  asm("s_nop 1\n" SRBD_FMAC11(K) SRBD_ASM_TAIL                                                        \
      : "+v"(S[a]), "+v"(S[b]), "+v"(S[c]), "+v"(S[d]), "+v"(S[e]), "+v"(S[f]), "+v"(S[g]), "+v"(S[h]), \
        "+v"(S[i]), "+v"(S[j]), "+v"(S[l])                                                          \
      : "v"(t))
__device__ __forceinline__ void pivot_update(double (&S)[12], double t, int k) {
  switch (k) {
    case 0: SRBD_PIVOT11(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11); break;
    case 1: SRBD_PIVOT11(1, 0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11); break;
    case 2: SRBD_PIVOT11(2, 0, 1, 3, 4, 5, 6, 7, 8, 9, 10, 11); break;
    case 3: SRBD_PIVOT11(3, 0, 1, 2, 4, 5, 6, 7, 8, 9, 10, 11); break;
    case 4: SRBD_PIVOT11(4, 0, 1, 2, 3, 5, 6, 7, 8, 9, 10, 11); break;
    case 5: SRBD_PIVOT11(5, 0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 11); break;
    case 6: SRBD_PIVOT11(6, 0, 1, 2, 3, 4, 5, 7, 8, 9, 10, 11); break;
    case 7: SRBD_PIVOT11(7, 0, 1, 2, 3, 4, 5, 6, 8, 9, 10, 11); break;
    case 8: SRBD_PIVOT11(8, 0, 1, 2, 3, 4, 5, 6, 7, 9, 10, 11); break;
    case 9: SRBD_PIVOT11(9, 0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 11); break;
    case 10: SRBD_PIVOT11(10, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 11); break;
    default: SRBD_PIVOT11(11, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10); break;
  }
}

// sum_j c[j] * v(lane j) over the 12 rows of a 16-lane DPP row (three interleaved accumulators)
__device__ __forceinline__ double dot_bc12(const double (&c)[12], double v) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  asm("s_nop 1\n"
      SRBD_FMAC_BC("%0", "%3", "%4", 0) SRBD_FMAC_BC("%1", "%3", "%5", 1) SRBD_FMAC_BC("%2", "%3", "%6", 2)
      SRBD_FMAC_BC("%0", "%3", "%7", 3) SRBD_FMAC_BC("%1", "%3", "%8", 4) SRBD_FMAC_BC("%2", "%3", "%9", 5)
      SRBD_FMAC_BC("%0", "%3", "%10", 6) SRBD_FMAC_BC("%1", "%3", "%11", 7) SRBD_FMAC_BC("%2", "%3", "%12", 8)
      SRBD_FMAC_BC("%0", "%3", "%13", 9) SRBD_FMAC_BC("%1", "%3", "%14", 10) SRBD_FMAC_BC("%2", "%3", "%15", 11)
      SRBD_ASM_TAIL
      : "+v"(a0), "+v"(a1), "+v"(a2)
      : "v"(v), "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]), "v"(c[5]), "v"(c[6]), "v"(c[7]),
        "v"(c[8]), "v"(c[9]), "v"(c[10]), "v"(c[11]));
  return (a0 + a1) + a2;
}

// Row r of the INVERSE of a 12x12 SPD block held one row per lane (row r = lane & 15 of a 16-lane
// DPP row, lanes 12..15 shadowing row 11; the chains run on lanes 0..31), by Gauss-Jordan pivoting
// on the diagonal. The pivot row is not rescaled in place (a plain sweep would multiply every
// element of every row by a select to special-case it): every lane keeps its row unscaled together
// with a scale factor (1/pivot once the row has been the pivot) that is applied once at the end, so
// each pivot costs one fused broadcast-FMA per element and lane (pivot_update).
//   pivot k (pk = row k, broadcast by row_newbcast inside the FMAs, id = 1/pk[k] by rcp3):
//     lane r != k: a_rj <- a_rj - a_rk id pk_j  (j != k),  a_rk <- a_rk id
//     lane k     : row unchanged except a_kk <- -1, scale <- id
// The pivot lanes of step k are a compile-time lane set, so their special cases are exec-masked
// 64-bit moves (2 SALU + 1 VALU each) instead of 64-bit selects (2 v_cndmask_b32 each): a_kk is
// zeroed on them right after the broadcast (t = a_kk id = 0 makes their update a no-op), then set
// to -1 with scale <- id after the update.
// On exit Dr[j] = (A^-1)_rj.
template <int K>
struct PivotLanes {  // s_and_saveexec_b64 literal (32-bit, sign-extended; lanes >= 32 are inactive)
  static constexpr uint32_t m16 = (1u << K) | (K == 11 ? 0xF000u : 0u);
  static constexpr int64_t value = (int32_t)(m16 | (m16 << 16));
};

template <int K>
__device__ __forceinline__ void gj_pivot(double (&Sr)[12], double& sc) {
  const double pk = bc16(Sr[K], K);
  uint64_t sv;
  asm("s_and_saveexec_b64 %[sv], %[m]\n\tv_mov_b64 %[x], 0\n\ts_mov_b64 exec, %[sv]"
      : [x] "+v"(Sr[K]), [sv] "=&s"(sv)
      : [m] "n"(PivotLanes<K>::value));
  const double id = rcp3(pk);
  const double t = Sr[K] * id;  // 0 on the pivot lanes
  pivot_update(Sr, t, K);       // Sr[j] -= pk[j] t, j != K
  Sr[K] = t;
  asm("s_and_saveexec_b64 %[sv], %[m]\n\tv_mov_b64 %[x], -1.0\n\tv_mov_b64 %[s], %[id]\n\ts_mov_b64 exec, %[sv]"
      : [x] "+v"(Sr[K]), [s] "+v"(sc), [sv] "=&s"(sv)
      : [id] "v"(id), [m] "n"(PivotLanes<K>::value));
  if constexpr (K < 11) gj_pivot<K + 1>(Sr, sc);
}

// The same sweep software-pipelined across pivots (bit-identical: every value is formed by the same
// operations in the same order). Pivot k+1's element a_{k+1,k+1} is final as soon as pivot k has
// updated column k+1, so that column's broadcast-FMA goes first; pivot k+1's broadcast and
// v_rcp_f64 then issue before pivot k's other ten broadcast-FMAs, which cover their latency, and
// the Newton step and t follow them. In the serial order every pivot waits on DPP -> rcp -> 2 FMA ->
// mul after its predecessor's last FMA. Where a partner wave hides that latency (one-wave QPs, two
// per SIMD) the split asm blocks cost more than they save (round 2: N = 10 +0.8 %); a two-wave QP's
// chain runs alone on its SIMD (its partner there is another QP's idle wave), where it pays.
#define SRBD_PIVOT1(K, a) asm("s_nop 1\n" SRBD_FMAC_BC("%0", "%0", "-%1", K) "s_nop 1\n" : "+v"(S[a]) : "v"(t))
#define SRBD_FMAC10(K)                                                                              \
  SRBD_FMAC_BC("%0", "%0", "-%10", K) SRBD_FMAC_BC("%1", "%1", "-%10", K) SRBD_FMAC_BC("%2", "%2", "-%10", K) \
  SRBD_FMAC_BC("%3", "%3", "-%10", K) SRBD_FMAC_BC("%4", "%4", "-%10", K) SRBD_FMAC_BC("%5", "%5", "-%10", K) \
  SRBD_FMAC_BC("%6", "%6", "-%10", K) SRBD_FMAC_BC("%7", "%7", "-%10", K) SRBD_FMAC_BC("%8", "%8", "-%10", K) \
  SRBD_FMAC_BC("%9", "%9", "-%10", K)
#define SRBD_PIVOT10(K, a, b, c, d, e, f, g, h, i, j)                                                \
  asm("s_nop 1\n" SRBD_FMAC10(K) SRBD_ASM_TAIL                                                       \
      : "+v"(S[a]), "+v"(S[b]), "+v"(S[c]), "+v"(S[d]), "+v"(S[e]), "+v"(S[f]), "+v"(S[g]), "+v"(S[h]), \
        "+v"(S[i]), "+v"(S[j])                                                                     \
      : "v"(t), "v"(y))
// pivot k's update of column k + 1 alone (its trailing s_nop 1: the next pivot's broadcast reads it)
__device__ __forceinline__ void pivot_update_next(double (&S)[12], double t, int k) {
  switch (k) {
    case 0: SRBD_PIVOT1(0, 1); break;
    case 1: SRBD_PIVOT1(1, 2); break;
    case 2: SRBD_PIVOT1(2, 3); break;
    case 3: SRBD_PIVOT1(3, 4); break;
    case 4: SRBD_PIVOT1(4, 5); break;
    case 5: SRBD_PIVOT1(5, 6); break;
    case 6: SRBD_PIVOT1(6, 7); break;
    case 7: SRBD_PIVOT1(7, 8); break;
    case 8: SRBD_PIVOT1(8, 9); break;
    case 9: SRBD_PIVOT1(9, 10); break;
    default: SRBD_PIVOT1(10, 11); break;
  }
}
// ... and of the ten columns other than k, k + 1 (y, the next pivot's raw reciprocal, is an unused
// operand: it pins the broadcast and v_rcp_f64 that produce it in front of the ten FMAs, which the
// scheduler would otherwise sink behind them)
__device__ __forceinline__ void pivot_update_rest(double (&S)[12], double t, double y, int k) {
  switch (k) {
    case 0: SRBD_PIVOT10(0, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11); break;
    case 1: SRBD_PIVOT10(1, 0, 3, 4, 5, 6, 7, 8, 9, 10, 11); break;
    case 2: SRBD_PIVOT10(2, 0, 1, 4, 5, 6, 7, 8, 9, 10, 11); break;
    case 3: SRBD_PIVOT10(3, 0, 1, 2, 5, 6, 7, 8, 9, 10, 11); break;
    case 4: SRBD_PIVOT10(4, 0, 1, 2, 3, 6, 7, 8, 9, 10, 11); break;
    case 5: SRBD_PIVOT10(5, 0, 1, 2, 3, 4, 7, 8, 9, 10, 11); break;
    case 6: SRBD_PIVOT10(6, 0, 1, 2, 3, 4, 5, 8, 9, 10, 11); break;
    case 7: SRBD_PIVOT10(7, 0, 1, 2, 3, 4, 5, 6, 9, 10, 11); break;
    case 8: SRBD_PIVOT10(8, 0, 1, 2, 3, 4, 5, 6, 7, 10, 11); break;
    case 9: SRBD_PIVOT10(9, 0, 1, 2, 3, 4, 5, 6, 7, 8, 11); break;
    default: SRBD_PIVOT10(10, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9); break;
  }
}
// pivot lanes of step K: a_KK <- 0 (so t = a_KK id is 0 there and their update is a no-op)
template <int K>
__device__ __forceinline__ void pivot_zero(double& x) {
  uint64_t sv;
  asm("s_and_saveexec_b64 %[sv], %[m]\n\tv_mov_b64 %[x], 0\n\ts_mov_b64 exec, %[sv]"
      : [x] "+v"(x), [sv] "=&s"(sv)
      : [m] "n"(PivotLanes<K>::value));
}
// pivot lanes of step K after the update: a_KK <- -1, scale <- id
template <int K>
__device__ __forceinline__ void pivot_finish(double& x, double& sc, double id) {
  uint64_t sv;
  asm("s_and_saveexec_b64 %[sv], %[m]\n\tv_mov_b64 %[x], -1.0\n\tv_mov_b64 %[s], %[id]\n\ts_mov_b64 exec, %[sv]"
      : [x] "+v"(x), [s] "+v"(sc), [sv] "=&s"(sv)
      : [id] "v"(id), [m] "n"(PivotLanes<K>::value));
}
// step K of the pipelined sweep, entered with pivot K's reciprocal id and multiplier t formed
template <int K>
__device__ __forceinline__ void gj_pivot_swp(double (&Sr)[12], double& sc, double id, double t) {
  if constexpr (K < 11) {
    pivot_update_next(Sr, t, K);               // column K + 1 first: a_{K+1,K+1} is now final
    const double pk = bc16(Sr[K + 1], K + 1);  // pivot K + 1's element ...
    const double y = __builtin_amdgcn_rcp(pk);  // ... and its raw reciprocal, in flight while
    pivot_update_rest(Sr, t, y, K);            // pivot K updates its ten other columns
    Sr[K] = t;
    pivot_finish<K>(Sr[K], sc, id);
    pivot_zero<K + 1>(Sr[K + 1]);
    const double e = fma(-pk, y, 1.0);
    const double idn = SRBD_RCP_NEWTON ? fma(y, e, y) : fma(y, fma(e, e, e), y);  // rcp3's step
    gj_pivot_swp<K + 1>(Sr, sc, idn, Sr[K + 1] * idn);
  } else {
    pivot_update(Sr, t, K);
    Sr[K] = t;
    pivot_finish<K>(Sr[K], sc, id);
  }
}
// kSwp: the software-pipelined sweep (same bits)
template <bool kSwp = false>
__device__ __forceinline__ void inverse_rows12(double (&Sr)[12], double (&Dr)[12]) {
  if constexpr (kSwp) {
    double sc = 1.0;
    const double pk = bc16(Sr[0], 0);
    pivot_zero<0>(Sr[0]);
    const double id = rcp3(pk);
    gj_pivot_swp<0>(Sr, sc, id, Sr[0] * id);
    const double nsc = -sc;
#pragma unroll
    for (int j = 0; j < 12; ++j) Dr[j] = Sr[j] * nsc;
    return;
  }
  double sc = 1.0;
  gj_pivot<0>(Sr, sc);
  // the sweep leaves -(A^-1) (times the row scale): flip the sign while applying the scale
  const double nsc = -sc;
#pragma unroll
  for (int j = 0; j < 12; ++j) Dr[j] = Sr[j] * nsc;
}

}  // namespace srbd
