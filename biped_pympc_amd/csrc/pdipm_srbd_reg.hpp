// pdipm_srbd_reg.hpp -- register-resident variant of the stage-invariant PDIPM kernel.
//
// Same algorithm, inputs and outputs as pdipm_srbd_kernel (pdipm_srbd.hpp; reference
// biped_pympc/casadi/sparse_pdipm_solver.py:357-534), re-laid out so that one QP needs <= 20 KiB of
// LDS at N = 10 and a CU holds 8 QPs = 2 waves per SIMD (the one-wave-per-SIMD kernel spends ~43% of
// its wave cycles parked on LDS latency; profiles/r01/). What moved out of LDS:
//   * the inequality-indexed vectors s, w = z/s + delta, D^-1 = 1/(1 + delta w), ds, dz, r_s live in
//     registers of the lane that owns row q = lane + 64 t (z keeps an LDS mirror for G^T z);
//   * the x-column part of r_x and the dynamics part of r_e live in registers of their owner lane;
//   * M (24 nonzeros), C = M diag(P / phi_x) (24, plus its pi-permuted transpose for the backward
//     group) and G (16 rows x 4 foot columns) are stored compactly;
//   * the two 4x4 foot inverses of Phi_u stay in the registers of their task lane;
//   * the block-recursion exchanges (rows of V = D^-1 C^T, the backward group's middle term, the
//     middle-vector hand-offs) go through DPP / ds_bpermute instead of LDS scratch, and the solve
//     chains keep w / v in registers (horizon is compile-time, chains fully unrolled).
// Compact M layout (same for C): [0..11] diag, [12 + 3r + k] = (r, 6 + k) for r < 3,
// [21 + r - 3] = (r, r + 6) for 3 <= r < 6 -- exactly the stage-coupling sparsity of -A_d.
#pragma once
#include "pdipm_srbd.hpp"
#include "qp_former.hpp"
#include "mpc_io.hpp"

#ifndef SRBD_PROGRESS_PRIO
#define SRBD_PROGRESS_PRIO 1  // progress-ordered wave priority (A/B switch for scripts/variant_bench.py)
#endif
#ifndef SRBD_PHASE_ATTR
#define SRBD_PHASE_ATTR  // diagnostic builds: __attribute__((noinline)) to read one phase ISA alone
#endif
#ifndef SRBD_REFINE_COMBINED
// the combined direction's refinement: 0 every iteration (product); diagnostic builds only: 1 never, 2 the
// last ceil(K / 2) iterations, 3 the dual rows (KKT row 4) only -- each measured faster (-16 / -8 / -3 % at
// N = 10) and each failing several times more parity-campaign cases (round 6)
#define SRBD_REFINE_COMBINED 0
#endif
#ifndef SRBD_SWP_INV
#define SRBD_SWP_INV 0  // two-wave QPs invert their chain blocks by the software-pipelined sweep: measured slower, off
#endif

namespace srbd {

// Threads per QP: one wave at N <= 10 (LDS and registers allow 2 QPs per SIMD); two waves beyond
// (the LDS of a longer horizon allows 1 QP per SIMD, so a second wave of the SAME QP takes the other
// half of every row-parallel phase and gives the SIMD a partner to hide latency behind); three from
// N = 22, four from N = 25 (2 QPs per CU by LDS either way: 8 waves per CU instead of 6, and two
// inequality-row slots per lane instead of the three that spilled 6-30 VGPRs at 192 threads). The
// block chains and the per-stage tasks stay on wave 0.
__host__ __device__ constexpr int reg_tpb(int N) { return N <= 10 ? 64 : (N <= 21 ? 128 : (N <= 24 ? 192 : 256)); }
// Horizons the register kernels are instantiated for: the equality-row slots need 6 N <= threads
// per QP (one wave to N = 10, two to N = 21, three or four to N = 32) and the fused prologue's 17 inputs fit
// the DV blocks from N = 2. N = 10 lives in srbd_mpc.hip, N = 20 in srbd_reg20.hip, the others in
// srbd_regN.hip; N = 1 runs the LDS-resident kernels.
__host__ __device__ constexpr bool reg_horizon(int N) { return N >= 2 && N <= 32; }

// Ordering of LDS accesses between the threads of one QP. A two-wave QP (N = 20) needs the
// workgroup barrier. A one-wave QP needs no wait at all: LDS operations of one wavefront are
// performed in order (AMDGPU memory model: s_waitcnt lgkmcnt(0) synchronises LDS between
// wavefronts of a workgroup, not within one), so a wavefront-scope fence -- a code-motion barrier
// that emits no s_waitcnt -- orders a phase's LDS writes before the next phase's reads. (A
// one-wave __syncthreads drains every outstanding LDS operation at each phase boundary.)
template <int TPB>
__device__ __forceinline__ void qp_sync() {
  if constexpr (TPB > 64) {
    __syncthreads();
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// LDS bank spreading of the stage-invariant blocks (a ds_read_b64 serves 32 lanes per pass from 64
// 4-byte banks): the u-block N is stored with row stride kNdS = 13, so the lanes of a row-parallel
// pass reading rows {0,1,2,6,7,8} (or all 12 rows, S_ii) of one column hit 12 distinct bank pairs
// (stride 12: rows r and r + 8 share a bank); G's foot-1 rows start kGfPad = 4 doubles after foot 0's
// (g_row), so the 8 lanes of a stage reading one row of both feet in G^T z use 16 distinct banks.
constexpr int kNdS = 13, kGfPad = 4, kGfSize = 64 + kGfPad;
__host__ __device__ constexpr int nd_idx(int r, int c) { return r * kNdS + c; }

template <int N, int TPB = reg_tpb(N)>
struct RegLayout {
  static constexpr int nz = 24 * N, m = 16 * N, p = 14 * N, nx = 12 * N;
  static constexpr int Mc = 0, Cc = Mc + 24, Nd = Cc + 48, Gf = Nd + 12 * kNdS, K0 = Gf + kGfSize, K1 = K0 + 78,
                       Pd = K1 + 78, IX = Pd + 12, Hu = IX + 12, SG = Hu + 24, TRI = SG + 16,
                       DV = TRI + 10,
                       X = DV + 80 * N,  // stage blocks of 80 doubles (78 used, kDvSlot)
                       Z = X + nz, Y = Z + m, RXu = Y + p, VV = RXu + nx, TV = VV + m,
                       QV = TV + nz, REm = QV + nx, DYm = REm + 2 * N,
                       RED = DYm + 2 * N,  // block reductions of a multi-wave QP: 2 slot sets
                       DMY = RED + (TPB > 64 ? 2 * (TPB / 64) : 0),  // sink of the invalid lanes' stores
                       end0 = DMY + 2,
                       // the fused prologue's FormerLds scratch from TV on (pads the short horizons)
                       former = TV + 2 * (int)((sizeof(FormerLds) + 15) / 16);
  static constexpr int end = end0, total = end > former ? end : former;
  // SE: the three equality-row register slots of RegCtx::erow (dynamics rows {0,1,2,6,7,8} and
  // {3,4,5,9,10,11} of every stage, then the x-moment rows), whatever the horizon
  static constexpr int SI = (m + TPB - 1) / TPB, SE = 3, SX = (nx + TPB - 1) / TPB;
  static_assert((DV & 1) == 0 && (X & 1) == 0 && (TV & 1) == 0, "16-byte aligned vectors");
};

// Index arithmetic on lane-derived values (non-negative, far below 2^16) through the full-rate
// 24-bit multiplier: the compiler cannot bound an opaque lane to 24 bits, so it emits the
// quarter-rate v_mul_lo_u32 / v_mul_hi_u32 for c / 12, 12 i and the like.
__device__ __forceinline__ int m24(int a, int b) { return (int)__umul24((unsigned)a, (unsigned)b); }
// c / 12 and c / 6 by reciprocal multiplication: 43691 * 12 = 2^19 + 4, exact for 0 <= c < 2^17
// (c / 6: < 2^16, where the product also stays below 2^32)
__device__ __forceinline__ int div12(int c) { return (int)(__umul24((unsigned)c, 43691u) >> 19); }
__device__ __forceinline__ int div6(int c) { return (int)(__umul24((unsigned)c, 43691u) >> 18); }

// foot of u column j ({0,1,2,7} left, {3,4,5,10} right, else -1), its position, and the inverse
__device__ __forceinline__ int foot_of(int j) { return (j < 3 || j == 7) ? 0 : ((j < 6 || j == 10) ? 1 : -1); }
__device__ __forceinline__ int foot_pos(int j) { return j < 6 ? j % 3 : 3; }
__host__ __device__ constexpr int foot_colj(int f, int a) { return a < 3 ? a + 3 * f : 7 + 3 * f; }
__host__ __device__ constexpr int perm12c(int j) { return j < 6 ? j + 6 : j - 6; }

// Block position of stage i inside DV: the forward group's step t (stage t) at 2t, the backward
// group's step t (stage N-1-t) at 2t+1, the middle stage at N-1. A step's two blocks then sit at
// 1248 t + 624 g bytes, so with the group term folded into the lane's offsets every block access of
// the chains is a fixed VGPR + an immediate offset (no per-step address arithmetic).
template <int N>
__host__ __device__ constexpr int dv_pos(int i) {
  return i < N / 2 ? 2 * i : (i == N / 2 ? N - 1 : 2 * (N - 1 - i) + 1);
}
// One symmetric 12x12 stage block: 78 distinct elements in 80 double slots. The slot of element
// (r, c) = (c, r) is kDvSlot[packed index r(r+1)/2 + c] (scripts/dv_slots.py): in every column the
// 12 rows sit in distinct slots mod 16, and the two twisted groups' blocks of a step are 80 doubles
// (= 16 mod 32) apart, so the 24 lanes of a chain load or store hit 24 distinct LDS bank pairs
// (the packed layout with stride 78 averaged 2.4 bank cycles per access). Every access to a block
// goes through this map: the per-lane offset tables below and the S_ii build's entry slots.
constexpr int kDvStride = 80;
constexpr int kDvBytes = kDvStride * 8;
constexpr uint8_t kDvSlot[78] = {77, 58, 32, 73, 46, 5,  52, 54, 50, 65, 53, 75, 31, 14, 76, 30, 69, 71, 64, 20,
                                 15, 48, 8,  3,  9,  23, 28, 21, 6,  49, 43, 44, 29, 18, 78, 51, 19, 61, 42, 79,
                                 41, 24, 33, 39, 70, 55, 2,  22, 37, 40, 67, 27, 26, 68, 60, 66, 57, 36, 59, 1,
                                 45, 74, 56, 0,  63, 7,  11, 12, 72, 10, 35, 25, 4,  16, 34, 62, 38, 13};
static __constant__ uint8_t c_dvslot[78] = {77, 58, 32, 73, 46, 5,  52, 54, 50, 65, 53, 75, 31, 14, 76, 30,
                                            69, 71, 64, 20, 15, 48, 8,  3,  9,  23, 28, 21, 6,  49, 43, 44,
                                            29, 18, 78, 51, 19, 61, 42, 79, 41, 24, 33, 39, 70, 55, 2,  22,
                                            37, 40, 67, 27, 26, 68, 60, 66, 57, 36, 59, 1,  45, 74, 56, 0,
                                            63, 7,  11, 12, 72, 10, 35, 25, 4,  16, 34, 62, 38, 13};


// Byte offset, inside a step's block pair, of element (row r, column c) of chain lane l (group
// g = l >> 4, row r = min(l & 15, 11), both in the group's coordinates): packed-lower slot of
// (pi^g r, pi^g c) + 624 g. One row of 12 per lane, read once per phase instead of recomputed.
struct ChainOffs {
  uint32_t o[32][12];
};
constexpr int sym_idx_c(int a, int b) { return a >= b ? a * (a + 1) / 2 + b : b * (b + 1) / 2 + a; }
constexpr ChainOffs make_chain_offs() {
  ChainOffs t{};
  for (int l = 0; l < 32; ++l) {
    const int g = l >> 4, r = (l & 15) < 12 ? (l & 15) : 11;
    const int pr = g ? perm12c(r) : r;
    for (int c = 0; c < 12; ++c)
      t.o[l][c] = (uint32_t)(8 * kDvSlot[sym_idx_c(pr, g ? perm12c(c) : c)] + kDvBytes * g);
  }
  return t;
}
static __constant__ ChainOffs c_choffs = make_chain_offs();

// this chain lane's 12 offsets (three 16-byte loads from the constant table)
__device__ __forceinline__ void load_chain_offs(int lane, uint32_t (&offs)[12]) {
  const uint4* p = reinterpret_cast<const uint4*>(c_choffs.o[lane & 31]);
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const uint4 v = p[q];
    offs[4 * q] = v.x;
    offs[4 * q + 1] = v.y;
    offs[4 * q + 2] = v.z;
    offs[4 * q + 3] = v.w;
  }
}
// double at DV byte offset off + imm (imm compile-time: folded into the ds instruction)
__device__ __forceinline__ double& dv_at(double* DV, uint32_t off, int imm) {
  return *reinterpret_cast<double*>(reinterpret_cast<char*>(DV) + off + imm);
}
// Reads are volatile so the compiler keeps them single ds_read_b64 (2 LDS cycles, conflict-free by
// the slot map) instead of pairing two blocks' elements into ds_read2_b64 (8 LDS cycles on gfx950,
// MI355X_MICROARCH.md LDS table)
typedef const volatile __attribute__((address_space(3))) double* lds_vcd_ptr;
__device__ __forceinline__ double dv_at(const double* DV, uint32_t off, int imm) {
  return *(lds_vcd_ptr)(reinterpret_cast<const char*>(DV) + off + imm);
}

// lane i of every 16-lane row <- lane i + 6 (rows 3..5 fetch rows 9..11)
__device__ __forceinline__ double shl6(double v) { return __builtin_amdgcn_mov_dpp(v, 0x106, 0xF, 0xF, true); }

// acc[i] += v[i](lane 6) c6 + v[i](lane 7) c7 + v[i](lane 8) c8 for 4 elements (the rows 6..8 term
// of the Schur update X = C V); kNeg: acc[i] -= the same
#define SRBD_ROWS678_4(N6, N7, N8)                                                                  \
  asm("s_nop 1\n"                                                                                   \
      SRBD_FMAC_BC("%0", "%4", N6, 6) SRBD_FMAC_BC("%1", "%5", N6, 6) SRBD_FMAC_BC("%2", "%6", N6, 6) \
      SRBD_FMAC_BC("%3", "%7", N6, 6) SRBD_FMAC_BC("%0", "%4", N7, 7) SRBD_FMAC_BC("%1", "%5", N7, 7) \
      SRBD_FMAC_BC("%2", "%6", N7, 7) SRBD_FMAC_BC("%3", "%7", N7, 7) SRBD_FMAC_BC("%0", "%4", N8, 8) \
      SRBD_FMAC_BC("%1", "%5", N8, 8) SRBD_FMAC_BC("%2", "%6", N8, 8) SRBD_FMAC_BC("%3", "%7", N8, 8) \
      SRBD_ASM_TAIL                                                                                   \
      : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)                                                      \
      : "v"(v0), "v"(v1), "v"(v2), "v"(v3), "v"(c6), "v"(c7), "v"(c8))
template <bool kNeg = false>
__device__ __forceinline__ void fmac_rows678_4(double& x0, double& x1, double& x2, double& x3, double v0,
                                               double v1, double v2, double v3, double c6, double c7,
                                               double c8) {
  if constexpr (kNeg)
    SRBD_ROWS678_4("-%8", "-%9", "-%10");
  else
    SRBD_ROWS678_4("%8", "%9", "%10");
}

// lane i of every 16-lane row <- lane i - 6 (rows 9..11 fetch rows 3..5)
__device__ __forceinline__ double shr6(double v) { return __builtin_amdgcn_mov_dpp(v, 0x116, 0xF, 0xF, true); }

// V = D^-1 C^T row by row: V[c] = Dr[c] C[c][c] + (c < 3: sum_k Dr[6 + k] C[c][6 + k])
// + (3 <= c < 6: Dr[c + 6] C[c][c + 6]), the coefficients of row c broadcast from lane c, which
// holds C's row c as (d, a0, a1, a2, b)
// Three blocks (rows 0..2, 3..5, 6..11) rather than one per row: the accumulator chains of a
// block's rows interleave (each FMA's accumulator was written 2-5 instructions earlier, not by the
// previous one), and two leading s_nop instead of eleven
__device__ __forceinline__ void v_rows(double (&V)[12], const double (&Dr)[12], double d, double a0, double a1,
                                       double a2, double b) {
  asm("s_nop 1\n"
      SRBD_FMAC_BC("%0", "%6", "%10", 0) SRBD_FMAC_BC("%1", "%6", "%11", 1) SRBD_FMAC_BC("%2", "%6", "%12", 2)
      SRBD_FMAC_BC("%0", "%7", "%13", 0) SRBD_FMAC_BC("%1", "%7", "%13", 1) SRBD_FMAC_BC("%2", "%7", "%13", 2)
      SRBD_FMAC_BC("%0", "%8", "%14", 0) SRBD_FMAC_BC("%1", "%8", "%14", 1) SRBD_FMAC_BC("%2", "%8", "%14", 2)
      SRBD_FMAC_BC("%0", "%9", "%15", 0) SRBD_FMAC_BC("%1", "%9", "%15", 1) SRBD_FMAC_BC("%2", "%9", "%15", 2)
      SRBD_ASM_TAIL
      : "=&v"(V[0]), "=&v"(V[1]), "=&v"(V[2])
      : "0"(0.0), "1"(0.0), "2"(0.0), "v"(d), "v"(a0), "v"(a1), "v"(a2), "v"(Dr[0]), "v"(Dr[1]), "v"(Dr[2]),
        "v"(Dr[6]), "v"(Dr[7]), "v"(Dr[8]));
  asm("s_nop 1\n"
      SRBD_FMAC_BC("%0", "%6", "%8", 3) SRBD_FMAC_BC("%1", "%6", "%9", 4) SRBD_FMAC_BC("%2", "%6", "%10", 5)
      SRBD_FMAC_BC("%0", "%7", "%11", 3) SRBD_FMAC_BC("%1", "%7", "%12", 4) SRBD_FMAC_BC("%2", "%7", "%13", 5)
      SRBD_ASM_TAIL
      : "=&v"(V[3]), "=&v"(V[4]), "=&v"(V[5])
      : "0"(0.0), "1"(0.0), "2"(0.0), "v"(d), "v"(b), "v"(Dr[3]), "v"(Dr[4]), "v"(Dr[5]), "v"(Dr[9]),
        "v"(Dr[10]), "v"(Dr[11]));
  asm("s_nop 1\n"
      SRBD_FMAC_BC("%0", "%12", "%13", 6) SRBD_FMAC_BC("%1", "%12", "%14", 7) SRBD_FMAC_BC("%2", "%12", "%15", 8)
      SRBD_FMAC_BC("%3", "%12", "%16", 9) SRBD_FMAC_BC("%4", "%12", "%17", 10) SRBD_FMAC_BC("%5", "%12", "%18", 11)
      SRBD_ASM_TAIL
      : "=&v"(V[6]), "=&v"(V[7]), "=&v"(V[8]), "=&v"(V[9]), "=&v"(V[10]), "=&v"(V[11])
      : "0"(0.0), "1"(0.0), "2"(0.0), "3"(0.0), "4"(0.0), "5"(0.0), "v"(d), "v"(Dr[6]), "v"(Dr[7]), "v"(Dr[8]),
        "v"(Dr[9]), "v"(Dr[10]), "v"(Dr[11]));
}

// (C w)_r and (C^T y)_r of the compact stage coupling for one vector held one element per lane:
// C has the diagonal, rows 0..2 x columns 6..8 and (r, r + 6) for 3 <= r < 6, so each is a local
// product, one row shift and three broadcast-FMAs (instead of a dense 12-term broadcast dot).
//   C w  : d w_r + b w_{r+6} + a0 w_6 + a1 w_7 + a2 w_8     (a* nonzero for r < 3, b for 3 <= r < 6)
//   C^T y: d y_r + b y_{r-6} + a0 y_0 + a1 y_1 + a2 y_2     (a* nonzero for 6 <= r < 9, b for r >= 9)
struct CoupleRow {
  double d, b, a0, a1, a2;
};
// Both with two accumulators (short dependent paths); the forward form folds the subtraction from
// the right-hand side into its first FMA: base - C w, and C^T y. A DPP instruction must not read ANY
// VGPR -- its fmac accumulator included -- written in the 2 wait states before it (the rule LLVM's
// hazard recognizer applies to every DPP operand; scripts/dpp_hazard_check.py audits the final ISA),
// hence the s_nop 0 before an accumulator's second FMA.
__device__ __forceinline__ double couple_cw_sub(const CoupleRow& c, double w, double base) {
  double a1 = fma(-c.d, w, base);
  double a2 = -c.b * shl6(w);
  asm("s_nop 1\n" SRBD_FMAC_BC("%0", "%2", "-%3", 6) SRBD_FMAC_BC("%1", "%2", "-%4", 7)
      "s_nop 0\n" SRBD_FMAC_BC("%0", "%2", "-%5", 8) SRBD_ASM_TAIL
      : "+v"(a1), "+v"(a2)
      : "v"(w), "v"(c.a0), "v"(c.a1), "v"(c.a2));
  return a1 + a2;
}
__device__ __forceinline__ double couple_cty2(const CoupleRow& c, double y) {
  double a1 = c.d * y;
  double a2 = c.b * shr6(y);
  asm("s_nop 1\n" SRBD_FMAC_BC("%0", "%2", "%3", 0) SRBD_FMAC_BC("%1", "%2", "%4", 1)
      "s_nop 0\n" SRBD_FMAC_BC("%0", "%2", "%5", 2) SRBD_ASM_TAIL
      : "+v"(a1), "+v"(a2)
      : "v"(y), "v"(c.a0), "v"(c.a1), "v"(c.a2));
  return a1 + a2;
}
// init - sum_j c[j] v(lane j) over the 12 rows of a 16-lane DPP row: two accumulators (the
// broadcast-FMAs issue every 8 cycles, so each accumulator's FMAs are 16 cycles apart) and one add;
// an s_nop 0 after each pair keeps 2 wait states between an accumulator's write and its next DPP
// read (a third accumulator would cost 2 VGPRs the N = 20 kernels do not have)
__device__ __forceinline__ double dot_bc12_sub(const double (&c)[12], double v, double init) {
  double a0 = init, a1 = 0.0;
  asm("s_nop 1\n"
      SRBD_FMAC_BC("%0", "%2", "-%3", 0) SRBD_FMAC_BC("%1", "%2", "-%4", 1) "s_nop 0\n"
      SRBD_FMAC_BC("%0", "%2", "-%5", 2) SRBD_FMAC_BC("%1", "%2", "-%6", 3) "s_nop 0\n"
      SRBD_FMAC_BC("%0", "%2", "-%7", 4) SRBD_FMAC_BC("%1", "%2", "-%8", 5) "s_nop 0\n"
      SRBD_FMAC_BC("%0", "%2", "-%9", 6) SRBD_FMAC_BC("%1", "%2", "-%10", 7) "s_nop 0\n"
      SRBD_FMAC_BC("%0", "%2", "-%11", 8) SRBD_FMAC_BC("%1", "%2", "-%12", 9) "s_nop 0\n"
      SRBD_FMAC_BC("%0", "%2", "-%13", 10) SRBD_FMAC_BC("%1", "%2", "-%14", 11)
      SRBD_ASM_TAIL
      : "+v"(a0), "+v"(a1)
      : "v"(v), "v"(c[0]), "v"(c[1]), "v"(c[2]), "v"(c[3]), "v"(c[4]), "v"(c[5]), "v"(c[6]), "v"(c[7]),
        "v"(c[8]), "v"(c[9]), "v"(c[10]), "v"(c[11]));
  return a0 + a1;
}

// element (c, b) of a compact M / C block (c or b runtime)
__device__ __forceinline__ double cel(const double* cc, int c, int b) {
  if (b == c) return cc[c];
  if (c < 3 && b >= 6 && b < 9) return cc[12 + 3 * c + b - 6];
  if (c >= 3 && c < 6 && b == c + 6) return cc[21 + c - 3];
  return 0.0;
}
// (M v)_r and (M^T v)_j from the compact block. The row / column is lane-dependent, so the sparse
// extra terms are formed in every lane from clamped indices and added with a 0 / 1 weight (fma(w, x,
// a) is a + x or a exactly): nested divergent branches (two exec-mask round trips each) cost more
// than the few FMAs, and a select would let the compiler sink the loads back into branches
// (M v)_r for the rows of equality slot t (RegCtx::erow): slot 0 holds r in {0,1,2,6,7,8}, where
// rows 0..2 add the columns-6..8 block; slot 1 r in {3,4,5,9,10,11}, where rows 3..5 add (r, r + 6)
template <int t>
__device__ __forceinline__ double mrow_slot(const double* mc, int r, const double* v) {
  const double a = mc[r] * v[r];
  if constexpr (t == 0) {
    const int rr = r < 3 ? r : 0;
    const double x = (mc[12 + 3 * rr] * v[6] + mc[13 + 3 * rr] * v[7]) + mc[14 + 3 * rr] * v[8];
    return fma(r < 3 ? 1.0 : 0.0, x, a);
  } else {
    const int rr = r < 6 ? r : 3;
    const double x = mc[21 + rr - 3] * v[rr + 6];
    return fma(r < 6 ? 1.0 : 0.0, x, a);
  }
}
__device__ __forceinline__ double mcol(const double* mc, int j, const double* v) {
  const double a = mc[j] * v[j];
  const bool b6 = j >= 6 && j < 9, b9 = j >= 9;
  const int j6 = b6 ? j - 6 : 0, j9 = b9 ? j - 9 : 0;
  const double x6 = (mc[12 + j6] * v[0] + mc[15 + j6] * v[1]) + mc[18 + j6] * v[2];
  const double x9 = mc[21 + j9] * v[j9 + 3];
  return fma(b9 ? 1.0 : 0.0, x9, fma(b6 ? 1.0 : 0.0, x6, a));
}
// dense 12-term row product (N block; rows are lane-dependent, so no per-row sparsity)
__device__ __forceinline__ double drow12(const double* row, const double* v) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    a0 += row[j] * v[j];
    a1 += row[j + 4] * v[j + 4];
    a2 += row[j + 8] * v[j + 8];
  }
  return (a0 + a1) + a2;
}
// (N^T v)_col over the stage u-block's sparsity: rows {0,1,2,6,7,8} are dense, rows {3+p, 9+p}
// (p = col % 3) hold only the force columns col < 6 (srbd_constraints.py:83-142 through B_d; the
// stored zeros make the formula exact for every col); kForce = false skips them (col >= 6 known)
template <bool kForce = true>
__device__ __forceinline__ double ncol(const double* nd, int col, const double* v, int p) {
  double a0 = nd[nd_idx(0, col)] * v[0] + nd[nd_idx(1, col)] * v[1];
  double a1 = nd[nd_idx(2, col)] * v[2] + nd[nd_idx(6, col)] * v[6];
  double a2 = nd[nd_idx(7, col)] * v[7] + nd[nd_idx(8, col)] * v[8];
  if (kForce) {
    a0 += nd[nd_idx(3 + p, col)] * v[3 + p];
    a1 += nd[nd_idx(9 + p, col)] * v[9 + p];
  }
  return (a0 + a1) + a2;
}

// Structural nonzeros of a foot's 8 inequality rows k over its columns (fx, fy, fz, my)
// (srbd_constraints.py:193-222): every row has fz; rows 0,1 also fx, rows 2,3 fy, rows 4,5 my,
// rows 6,7 nothing else. g_other(k) is that other column's position (0 for rows 6,7, where G is a
// stored structural zero, so the formula stays uniform across lanes).
__host__ __device__ constexpr int g_other(int k) { return k < 2 ? 0 : (k < 4 ? 1 : (k < 6 ? 3 : 0)); }

// G rows in LDS: row k (= 8 f + k', foot f) at 4 k + kGfPad f (see kGfPad)
__host__ __device__ constexpr int g_row(int k) { return 4 * k + kGfPad * (k >> 3); }

// (G xu)_k over row k's structural nonzeros (fz and the other column)
__device__ __forceinline__ double grow4(const double* gf, int k, const double* xu) {
  const int f = k >> 3, o = g_other(k & 7);
  const double* g = gf + g_row(k);
  return g[o] * xu[foot_colj(f, o)] + g[2] * xu[foot_colj(f, 2)];
}

// kFReg: every entry of f, b and h this lane uses held in registers (the fused kernel, which computes
// them); false: f's slots t >= 1, b's x-moment slot and h's last slot are re-read from memory (L2)
// each iteration -- the CCS kernel, whose stage-invariance check, three iterate initialisations and
// fallback call leave no room for them: held, they spilled 2-4 VGPRs (scratch reloads in the loop)
template <int N, bool kFReg = true>
struct RegCtx {
  static constexpr int TPB = reg_tpb(N);
  using Lo = RegLayout<N>;
  static constexpr int nz = Lo::nz, m = Lo::m, p = Lo::p, nx = Lo::nx;
  static constexpr int SI = Lo::SI, SE = Lo::SE, SX = Lo::SX;
  // Equality rows by register slot: slot 0 holds the dynamics rows {0,1,2,6,7,8} of every stage (the
  // dense rows of the u-block N), slot 1 rows {3,4,5,9,10,11} (two force columns each), slot 2 the
  // x-moment rows, so each slot's row formula is the same in every lane.
  static_assert(6 * N <= TPB && 2 * N <= TPB, "equality-row slots");
  struct ERow {
    int e, i, r;
    bool valid;
  };
  __device__ static ERow erow(int l, int t) {
    ERow q;
    if (t == 2) {
      q.valid = l < 2 * N;
      q.e = nx + l;
      q.i = l >> 1;
      q.r = l & 1;
      return q;
    }
    q.valid = l < 6 * N;
    q.i = div6(l);
    const int k = l - m24(q.i, 6);
    q.r = t == 0 ? (k < 3 ? k : k + 3) : (k < 3 ? k + 3 : k + 6);
    q.e = m24(q.i, 12) + q.r;
    return q;
  }
  // (N u)_r of stage i's u block for a slot-t row (slot 1: the two force columns of row r)
  template <int t>
  __device__ static double nrow(const double* nd, int r, const double* u) {
    if constexpr (t == 0) {
      return drow12(nd + nd_idx(r, 0), u);
    } else {
      const int p = r % 3;
      return nd[nd_idx(r, p)] * u[p] + nd[nd_idx(r, 3 + p)] * u[3 + p];
    }
  }
  static constexpr int mid = N / 2, nf = mid, nb = N - 1 - mid, T = nf > nb ? nf : nb;
  // the chain's 12x12 block inverses by the software-pipelined sweep (inverse_rows12<true>), tried for
  // two-wave QPs on the premise that their chain wave runs alone on its SIMD (profiles/r05/simd_probe.txt:
  // its SIMD partner is another QP's second wave); measured +2.1 % at N = 20 (n20_pipeline.txt): off
  static constexpr bool kSwpInv = SRBD_SWP_INV && TPB == 128;
  static constexpr int kFactorUnroll = T + 1;  // chains fully unrolled (N = 20: -4.7 % vs rolled)
  double* L;
  int lane;
  // The CCS kernel's f, h, b rows of this env. At N = 21 they are addressed from the kernel's own
  // argument (kernarg segment: scalar loads) at each use: a 64-bit row pointer held across the Newton
  // loop is what that kernel spilled (a scratch reload per iteration). Elsewhere the three row
  // pointers are held (the per-use address arithmetic cost the N = 10 kernel ~1 %,
  // profiles/r05/ab_*.txt). tests/test_isa_hazards.py checks the choice at every horizon. Unused by the
  // fused kernel (kFReg).
  static constexpr bool kArgRows = N == 21;
  int env_ = 0;
  const double *fp_ = nullptr, *hp_ = nullptr, *bp_ = nullptr;
  __device__ const double* fg() const { return kArgRows ? solver_in(kernel_args(), 3) + (size_t)env_ * nz : fp_; }
  __device__ const double* hg() const { return kArgRows ? solver_in(kernel_args(), 4) + (size_t)env_ * m : hp_; }
  __device__ const double* bg() const { return kArgRows ? solver_in(kernel_args(), 5) + (size_t)env_ * p : bp_; }
  // this lane's entries of f (x and u columns), b and h, held in registers for the whole solve:
  // set once (loaded, or as the fused kernel computes them), never re-read from memory
  double fxr[SX], fur[SX], bvr[SE], hvr[SI];
  __device__ void load_qp_vectors() {
#pragma unroll
    for (int t = 0; t < (kFReg ? SX : 1); ++t) {
      const int c = min(lane + TPB * t, nx - 1);
      fxr[t] = fg()[c];
      fur[t] = fg()[nx + c];
    }
#pragma unroll
    for (int t = 0; t < (kFReg ? SE : 2); ++t) {
      const ERow q = erow(lane, t);
      bvr[t] = bg()[q.valid ? q.e : 0];
    }
#pragma unroll
    for (int t = 0; t < (kFReg ? SI : SI - 1); ++t) hvr[t] = hg()[min(lane + TPB * t, m - 1)];
  }
  // h of slot t (the CCS kernel re-reads its last slot from memory, see kFReg)
  __device__ double hval(int t, int q) const { return (kFReg || t < SI - 1) ? hvr[t] : hg()[q]; }
  // ph: this foot-task lane's LDL^T factors of its foot block Phi_f (foot_inverse, phi_solve)
  double s[SI], z[SI], wd[SI], di[SI], ds[SI], dz[SI], rs[SI], re[SE], rxx[SX], ph[10];
  double e3r[SI];  // the affine refinement's row-3 residuals (degenerate iterations only)
  PROF_DECL

  __device__ double* at(int off) const { return L + off; }
  // Sum / min over the QP's threads. One wave: a DPP wave reduction. Two waves: each wave reduces,
  // writes its partial to LDS, and after a barrier both combine the partials in the same order
  // (identical result in both waves). Consecutive reductions alternate slot pairs: a wave writes
  // pair k only after passing reduction k-1's barrier, i.e. after the other wave has read pair k.
  int red_k = 0;
  template <bool kMin>
  __device__ double block_reduce(double v) {
    v = kMin ? wave_min(v) : wave_sum(v);
    if constexpr (TPB > 64) {
      constexpr int NW = TPB / 64;
      double* R = at(Lo::RED) + NW * red_k;
      red_k ^= 1;
      if ((lane & 63) == 0) R[lane >> 6] = v;
      qp_sync<TPB>();
      v = R[0];
#pragma unroll
      for (int w = 1; w < NW; ++w) v = kMin ? fmin(v, R[w]) : v + R[w];
    }
    return v;
  }
  __device__ double block_sum(double v) { return block_reduce<false>(v); }
  // the QP's threads vote (wave-uniform result)
  __device__ bool block_any(bool p) {
    if constexpr (TPB == 64) return __any(p);
    else return block_reduce<true>(p ? 0.0 : 1.0) < 0.5;
  }
  // any(p) || all(q) over the QP's threads in one vote (one reduction for a multi-wave QP)
  __device__ bool block_any_or_all(bool p, bool q) {
    if constexpr (TPB == 64) return __any(p) || !__any(!q);
    else return block_reduce<true>(p ? -1.0 : (q ? 1.0 : 0.0)) != 0.0;
  }
  __device__ double block_min(double v) { return block_reduce<true>(v); }
  // The lane index, re-materialised as an opaque value at the start of every phase: keeps the
  // compiler from hoisting each phase's per-lane addresses and predicates out of the Newton loop
  // (that alone pinned > 100 registers for the whole solve).
  // Its upper bound stays known (l < TPB: guards of whole slots and lane ranges fold). Telling the
  // compiler l >= 0 as well (unsigned index divisions) makes the fused N = 10 kernel spill 12 VGPRs.
  __device__ int fresh_lane() const {
    int l = lane;
    asm volatile("" : "+v"(l));
    __builtin_assume(l < TPB);
    return l;
  }
  // Slot t of a row-parallel pass over n rows (row = lane + TPB t) lies wholly inside [0, n): its row
  // guard is then constant-true and compiles to nothing -- the opaque lane of fresh_lane() hides
  // lane < TPB from the compiler, which otherwise branches on every slot's guard
  __device__ static constexpr bool full_slot(int t, int n) { return TPB * (t + 1) <= n; }

  // --------------------------------------------------------------------- residuals ----
  // Equality-row slots run in every lane: a lane past the slot's rows (q.valid false) computes on
  // in-bounds LDS rows of a stage past the horizon, keeps the result in its own re[t] (read only
  // under q.valid) and stores to the DMY sink -- no divergent branch around the phase.
  // (A v)_r of one dynamics row: M v_{i-1} (stage 0 has none: weight 0) + P v_i + N u_i
  template <int t>
  __device__ double arow(const double* V, const double* Mc, const double* Pd, const double* Nd, const ERow& q) const {
    const double mv = mrow_slot<t>(Mc, q.r, V + 12 * (q.i >= 1 ? q.i - 1 : 0));
    double v = (q.i >= 1 ? 1.0 : 0.0) * mv;
    v += Pd[q.r] * V[12 * q.i + q.r];
    v += nrow<t>(Nd, q.r, V + nx + 12 * q.i);
    return v;
  }
  // index into the vector at L + base of row e, or the DMY sink for an invalid lane
  __device__ static int sink(bool valid, int e, int base) { return valid ? e : Lo::DMY - base; }
  template <int t>
  __device__ void re_slot(const double* X, const double* Mc, const double* Pd, const double* Nd,
                          const double (&bv)[SE]) {
    const ERow q = erow(fresh_lane(), t);
    re[t] = arow<t>(X, Mc, Pd, Nd, q) - bv[t];
  }
  template <int t>
  __device__ void g_slot(const double* TV, const double* Mc, const double* Pd, const double* Nd, double* QV) {
    const ERow q = erow(fresh_lane(), t);
    QV[sink(q.valid, q.e, Lo::QV)] = arow<t>(TV, Mc, Pd, Nd, q) + re[t];
  }
  // want_mu (wave-uniform): also return mu = s^T z / m -- the first iteration only: afterwards it
  // equals the previous iteration's mu_new, the same products s_t z_t summed in the same order
  SRBD_PHASE_ATTR __device__ double residuals(bool want_mu) {
    const int lane = fresh_lane();
    const double *X = at(Lo::X), *Y = at(Lo::Y), *Z = at(Lo::Z), *Mc = at(Lo::Mc), *Nd = at(Lo::Nd),
                 *Gf = at(Lo::Gf), *Pd = at(Lo::Pd), *Hu = at(Lo::Hu), *SG = at(Lo::SG);
    double *RXu = at(Lo::RXu), *REm = at(Lo::REm);
    const double(&fx)[SX] = fxr, (&fu)[SX] = fur, (&bv)[SE] = bvr, (&hv)[SI] = hvr;
#pragma unroll
    for (int t = 0; t < SX; ++t) {  // r_x, x columns: H_x x + f + P y_{k-1} + M^T y_k (owner regs)
      const int c = lane + TPB * t;
      if (full_slot(t, nx) || c < nx) {
        const int k = div12(c) + 1, j = c - m24(k - 1, 12);
        const double v = Hu[12 + j] * X[c] + ((kFReg || t == 0) ? fx[t] : fg()[c]);
        double ay = Pd[j] * Y[12 * (k - 1) + j];
        const double my = mcol(Mc, j, Y + 12 * (k < N ? k : N - 1));  // k = N: unused
        ay = fma(k < N ? 1.0 : 0.0, my, ay);
        rxx[t] = v + ay;
      }
    }
#pragma unroll
    for (int t = 0; t < SX; ++t) {  // r_x, u columns: H_u u + f + G^T z + N^T y + e-rows (LDS)
      const int c = lane + TPB * t;
      if (full_slot(t, nx) || c < nx) {
        const int i = div12(c), j = c - m24(i, 12);
        const double v = Hu[j] * X[nx + c] + ((kFReg || t == 0) ? fu[t] : fg()[nx + c]);
        // G^T z on the foot columns and the x-moment terms on columns 6 / 9, formed in every lane
        // (clamped foot index) and selected
        const int fj = foot_of(j), f = fj >= 0 ? fj : 0;
        const double* zf = Z + 16 * i + 8 * f;
        const double* g = Gf + g_row(8 * f) + foot_pos(j);
        double g0 = 0.0, g1 = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          g0 += g[4 * k] * zf[k];
          g1 += g[4 * (k + 4)] * zf[k + 4];
        }
        const double gz = (fj >= 0 ? 1.0 : 0.0) * (g0 + g1);
        double ay = ncol(Nd, j, Y + 12 * i, j % 3);
        const bool e9 = j == 9;
        const double se = (j == 6 || e9) ? 1.0 : 0.0;
        ay = fma(se * (e9 ? SG[7] : SG[6]), Y[nx + 2 * i + (e9 ? 1 : 0)], ay);
        RXu[c] = (v + gz) + ay;
      }
    }
    re_slot<0>(X, Mc, Pd, Nd, bv);  // r_e = A x - b (owner regs; x-moment rows also in LDS)
    re_slot<1>(X, Mc, Pd, Nd, bv);
    {
      const ERow q = erow(lane, 2);
      if (q.valid) {
        const int w = q.r;
        re[2] = SG[6 + w] * X[nx + 12 * q.i + (w ? 9 : 6)] - (kFReg ? bv[2] : bg()[q.e]);
        REm[q.e - nx] = re[2];
      }
    }
    double sz = 0.0;
#pragma unroll
    for (int t = 0; t < SI; ++t) {  // r_s = G u + s - h (owner regs)
      const int q = lane + TPB * t;
      if (RegCtx<N>::full_slot(t, m) || q < m) {
        const int i = q >> 4, k = q & 15;
        const double v = grow4(Gf, k, X + nx + m24(i, 12));
        rs[t] = (v + s[t]) - ((kFReg || t < SI - 1) ? hv[t] : hg()[q]);
        sz += s[t] * z[t];
      }
    }
    qp_sync<TPB>();
    return want_mu ? block_sum(sz) / m : 0.0;
  }

  // Right-hand side of forward elimination step t: g_i - C w_{i-1} (base = this lane's g_i entry),
  // and at the middle step also - C^T v_{mid+1} of group 1 (its lanes compute - C v with base 0
  // and hand it to group 0 through ds_bpermute)
  __device__ static double fwd_rhs(bool act, bool prev, bool mstep, int g, int r, const CoupleRow& Cr, double w,
                                   const double* qv) {
    double q = 0.0;
    if (act && !(mstep && g == 1)) q = *qv;
    if (act && prev) q = couple_cw_sub(Cr, w, q);
    if (mstep && nb >= 1) q += __shfl(q, 16 + perm12(r), 64);  // group 0 += group 1's - C^T v_{mid+1}
    return q;
  }

  // -------------------------------------------------------------------- factorise ----
  __device__ void factor() {
    factor_build();
    factor_chain<false>();
  }

  // The two 4x4 foot blocks of Phi_u = H_u + beta + G^T Lambda G of per-stage task fl = 2 i + f
  // (Lambda in VV), inverted; kept in this lane's registers (ph) and in dst[20 i + 10 f ..] for the
  // S_ii build
  __device__ void foot_inverse(int fl, double* dst) {
    const double *VV = at(Lo::VV), *Gf = at(Lo::Gf), *Hu = at(Lo::Hu);
    const int i = fl >> 1, f = fl & 1;
    double a[10];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c <= r; ++c) a[r * (r + 1) / 2 + c] = (r == c) ? Hu[foot_colj(f, r)] + kBeta : 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // + G_k^T lam_k G_k over row k's structural nonzeros
      const double lam = VV[16 * i + 8 * f + k];
      const double* g4 = Gf + g_row(8 * f + k);
      const double gz = g4[2];
      a[5] += lam * gz * gz;  // (fz, fz)
      if (k < 6) {
        const int o = g_other(k);  // fx, fy or my (k is unrolled: constant)
        const double go = g4[o];
        a[o * (o + 1) / 2 + o] += lam * go * go;
        if (o < 2) a[3 + o] += lam * gz * go;  // (fz, o)
        else a[8] += lam * go * gz;            // (my, fz)
      }
    }
    // LDL^T factors for the solves (ph: phi_solve) and, from them, the inverse for the S_ii build (dst):
    // the Schur complement and the solves take the same Phi_f^-1 (a mismatched pair -- the sweep
    // inverse in S_ii, stable solves in dx -- left z 1e-4 off at K = 20)
    ldlt_factor<4, true>(a);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double ec[4] = {c == 0 ? 1.0 : 0.0, c == 1 ? 1.0 : 0.0, c == 2 ? 1.0 : 0.0, c == 3 ? 1.0 : 0.0}, pc[4];
      ldlt_solve<4>(a, ec, pc);
#pragma unroll
      for (int r = c; r < 4; ++r) dst[20 * i + 10 * f + r * (r + 1) / 2 + c] = pc[r];
    }
#pragma unroll
    for (int e = 0; e < 10; ++e) ph[e] = a[e];
  }
  // x = Phi_f^-1 v for foot task fl, by a stable solve with the lane's LDL^T factors: the explicit
  // inverse applied to v loses the stiff direction G_i dx of rows with W = z / s ~ 1e7..1e8, whose error
  // Lambda ~ W multiplies into dz.
  __device__ void phi_solve(int fl, const double (&v)[4], double (&x)[4]) const {
    (void)fl;
    ldlt_solve<4>(ph, v, x);
  }

  // Phi_u foot inverses and the S_ii blocks (parallel over the wave)
  SRBD_PHASE_ATTR __device__ void factor_build() {
    const int lane = fresh_lane();
    double *VV = at(Lo::VV), *DV = at(Lo::DV), *PHs = at(Lo::TV);  // PHs: scratch, TV is dead here
    const double *Gf = at(Lo::Gf), *Hu = at(Lo::Hu), *Nd = at(Lo::Nd), *K0 = at(Lo::K0), *K1 = at(Lo::K1);
    const uint8_t* TRI = reinterpret_cast<const uint8_t*>(at(Lo::TRI));
#pragma unroll
    for (int t = 0; t < SI; ++t) {
      const int q = lane + TPB * t;
      if (RegCtx<N>::full_slot(t, m) || q < m) {
        wd[t] = rcp3(s[t]) * z[t] + kDelta;  // correctly rounded reciprocals (rcp3), not IEEE division
        di[t] = rcp3(1.0 + kDelta * wd[t]);
        VV[q] = di[t] * wd[t];  // Lambda, shared with the foot tasks
      }
    }
    qp_sync<TPB>();
    if (lane < 2 * N) foot_inverse(lane, PHs);
    qp_sync<TPB>();
    // S_ii = K + sum_f N_f Phi_f^-1 N_f^T in two divergence-free passes over the class-sorted entry
    // table (TRI = c_tab.dvo: 21 dense x dense entries, then 57 with a sparse index): an entry
    // touching rows {3,4,5,9,10,11} of N needs 10 FMAs instead of 40
    // Each lane keeps ONE entry (r, c) for the whole pass, so its table entry, N rows and K values
    // are loaded once; only Phi_f^-1 (PHs) changes with the stage.
    // with two waves each takes half of the stages: wave w's lane l < 63 -> class q = 3 w + l / 21
    constexpr int NW = TPB / 64, NQ = 3 * NW;
    const int lw = lane & 63, wv = lane >> 6;
    if (lw < 63) {  // dense x dense: lw = 21 q' + k -> entry k of stages NQ t + q, q = 3 wv + q'
      const int q = 3 * wv + lw / 21, k = lw - 21 * (lw / 21);
      const int rc = TRI[k], r = rc & 15, c = rc >> 4, sy = r * (r + 1) / 2 + c, sl = c_dvslot[sy];
      // n_r Phi^-1 n_c^T = sum over packed (a >= b) of Phi^-1_ab w_ab with the stage-invariant pair
      // products w_aa = n_ra n_ca, w_ab = n_ra n_cb + n_rb n_ca: 10 FMAs per foot and stage, not 20
      double w[2][10];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        double vr[4], vc[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          vr[a] = Nd[nd_idx(r, foot_colj(f, a))];
          vc[a] = Nd[nd_idx(c, foot_colj(f, a))];
        }
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b <= a; ++b)
            w[f][a * (a + 1) / 2 + b] = a == b ? vr[a] * vc[a] : vr[a] * vc[b] + vr[b] * vc[a];
      }
      const double k0 = K0[sy], k1 = K1[sy];
#pragma unroll
      for (int t = 0; t < (N + NQ - 1) / NQ; ++t) {
        const int i = NQ * t + q;
        if (i < N) {
          double v = i == 0 ? k0 : k1;
#pragma unroll
          for (int f = 0; f < 2; ++f) {
            const double* ph_ = PHs + 20 * i + 10 * f;
#pragma unroll
            for (int e = 0; e < 10; ++e) v += ph_[e] * w[f][e];
          }
          DV[kDvStride * dv_pos<N>(i) + sl] = v;
        }
      }
    }
    if (lw < 57) {  // the 57 entries with a sparse index (rows {3,4,5,9,10,11} of N hold one entry
                      // per foot, at position r % 3), one stage per trip; for a sparse x sparse entry
                      // the 4-term sum over the "dense" index meets N's zeros, so it is exact too
      const int rc = TRI[21 + lw], r = rc & 15, c = rc >> 4, sy = r * (r + 1) / 2 + c, sl = c_dvslot[sy];
      const bool rs = (r % 6) >= 3;
      const int sp = rs ? r : c, dn = rs ? c : r, as = sp % 3;
      double wn[2][4];  // stage-invariant products n_sp,as * n_dn,b: 4 FMAs per foot and stage
      int po[4];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const double ns = Nd[nd_idx(sp, foot_colj(f, as))];
#pragma unroll
        for (int b = 0; b < 4; ++b) wn[f][b] = ns * Nd[nd_idx(dn, foot_colj(f, b))];
      }
#pragma unroll
      for (int b = 0; b < 4; ++b) po[b] = sym_idx(as, b);
      const double k0 = K0[sy], k1 = K1[sy];
#pragma unroll 2
      // wave wv's share of the stages: [wv N / NW, (wv + 1) N / NW) (uneven when NW does not divide N)
      for (int i = (wv * N) / NW; i < ((wv + 1) * N) / NW; ++i) {
        double v = i == 0 ? k0 : k1;
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const double* ph_ = PHs + 20 * i + 10 * f;
#pragma unroll
          for (int b = 0; b < 4; ++b) v += ph_[po[b]] * wn[f][b];
        }
        DV[kDvStride * dv_pos<N>(i) + sl] = v;
      }
    }
    qp_sync<TPB>();
    PROF_ADD(1);
  }

  // kFwd: also the affine solve's forward elimination w_i = D_i^-1 (g_i - C w_{i-1}) with each
  // block's inverse row still in registers (g from solve_rhs(0) in QV; w_i written back over g_i)
  template <bool kFwd>
  SRBD_PHASE_ATTR __device__ void factor_chain() {
    const int lane = fresh_lane();
    double* DV = at(Lo::DV);
    double* QV = at(Lo::QV);
    // Twisted block recursion (see pdipm_srbd.hpp FastCtx::factor): group 0 (lanes 0..15) forward,
    // group 1 (lanes 16..31) backward in pi-permuted coordinates, middle block by group 0. Row r of
    // V = D^-1 Cg^T is computed by lane r; X = Cg V needs rows {r, 6, 7, 8} (r < 3) or {r, r + 6}
    // (3 <= r < 6), fetched with row_newbcast / row_shl:6 DPP; group 1's middle term reaches
    // group 0 through ds_bpermute.
    if (lane < 32) {
      const int g = lane >> 4, l16 = lane & 15;
      const int r = l16 < 12 ? l16 : 11;
      const int pr = g ? perm12(r) : r;
      const int cnt = g ? nb : nf;
      const double* cc = at(Lo::Cc) + 24 * g;
      // the coupling row's coefficients loaded from clamped indices and selected (a conditional
      // load is an exec-mask round trip per coefficient)
      const double crd = cc[r];
      const bool ra = r < 3, rb = r >= 3 && r < 6;
      const int r3 = ra ? r : 0, r6 = rb ? r : 3;
      const double la0 = cc[12 + 3 * r3], la1 = cc[13 + 3 * r3], la2 = cc[14 + 3 * r3], lb = cc[21 + r6 - 3];
      const double cra0 = ra ? la0 : 0.0, cra1 = ra ? la1 : 0.0, cra2 = ra ? la2 : 0.0;
      const double crb = rb ? lb : 0.0;
      uint32_t offs[12];  // byte offset of (pr, column c in group coordinates) in a step's blocks
      load_chain_offs(lane, offs);
      const CoupleRow Cr{crd, crb, cra0, cra1, cra2};
      double wf = 0.0;  // forward-elimination vector of the fused affine solve
      double Dr[12];
#pragma unroll
      for (int c = 0; c < 12; ++c) Dr[c] = 0.0;
#pragma unroll kFactorUnroll
      for (int t = 0; t <= T; ++t) {
        const bool mstep = (t == T);
        const int i = mstep ? mid : (g ? N - 1 - t : t);
        const bool act = mstep ? true : (t < cnt);
        const bool prev = mstep ? (cnt >= 1) : (t >= 1);
        double Sr[12], X[12];
#pragma unroll
        for (int c = 0; c < 12; ++c) X[c] = 0.0;
        const int imm = mstep ? kDvBytes * (N - 1) : 2 * kDvBytes * t;  // this step's blocks
        if (act) {
          if (!(mstep && g == 1)) {
#pragma unroll
            for (int c = 0; c < 12; ++c) Sr[c] = dv_at(DV, offs[c], imm);
          }
          if (prev) {
            double V[12];
            // V[c] = sum_k Dr[k] C[c][k]: row c of C is lane c's own coupling row (crd, cra*, crb),
            // broadcast inside the FMAs (row_newbcast:c) instead of re-read from LDS every step
            v_rows(V, Dr, crd, cra0, cra1, cra2, crb);
            if (!mstep) {  // S - X accumulated in place
#pragma unroll
              for (int c = 0; c < 12; ++c) Sr[c] = (Sr[c] - crd * V[c]) - crb * shl6(V[c]);
#pragma unroll
              for (int c = 0; c < 12; c += 4)  // - rows 6..8 of V through fused broadcast-FMAs
                fmac_rows678_4<true>(Sr[c], Sr[c + 1], Sr[c + 2], Sr[c + 3], V[c], V[c + 1], V[c + 2], V[c + 3],
                                     cra0, cra1, cra2);
            } else {  // middle step: group 1's X is handed to group 0 below
#pragma unroll
              for (int c = 0; c < 12; ++c) X[c] = crd * V[c] + crb * shl6(V[c]);
#pragma unroll
              for (int c = 0; c < 12; c += 4)  // + rows 6..8 of V through fused broadcast-FMAs
                fmac_rows678_4(X[c], X[c + 1], X[c + 2], X[c + 3], V[c], V[c + 1], V[c + 2], V[c + 3], cra0,
                               cra1, cra2);
              if (g == 0) {
#pragma unroll
                for (int c = 0; c < 12; ++c) Sr[c] -= X[c];
              }
            }
          }
        }
        if (mstep && nb >= 1) {  // X_b[r][c] = X'[pi r][pi c], held by lane 16 + pi(r)
#pragma unroll
          for (int c = 0; c < 12; ++c) {
            const double xb = __shfl(X[perm12c(c)], 16 + perm12(r), 64);
            if (g == 0) Sr[c] -= xb;
          }
        }
        if (act && !(mstep && g == 1)) {
          inverse_rows12<kSwpInv>(Sr, Dr);
          // every lane writes its whole row: (r, c) and (c, r) share a packed slot, so each slot is
          // written twice with the two (rounding-different) halves of the symmetric inverse; the
          // later ds_write in program order wins, deterministically (shadow lanes 12..15 repeat row
          // 11 bit for bit). Cheaper than 12 per-element exec-masked stores.
#pragma unroll
          for (int c = 0; c < 12; ++c) dv_at(DV, offs[c], imm) = Dr[c];
        }
        if constexpr (kFwd) {  // the solve chain's forward step t (solve_chain), Dr = D_i^-1 row
          const double q = fwd_rhs(act, prev, mstep, g, r, Cr, wf, QV + 12 * i + pr);
          if (act && !(mstep && g == 1)) {
            wf = dot_bc12(Dr, q);
            QV[12 * i + pr] = wf;  // shadow lanes 12..15 store row 11's value bit for bit
          }
        }
      }
    }
    qp_sync<TPB>();
    PROF_ADD(2);
  }

  // ------------------------------------------------------------------------ solve ----
  // kMode 0: affine rhs r2 = -(S^-1 (s o z)); 1: combined r2 = affine - S^-1 (s o z + ds o dz - smu).
  // One solve = solve_rhs (t = Phi^-1 r~ and the dual right-hand side g, in QV) -> solve_chain
  // (the twisted block forward elimination and back substitution: dy in QV) -> solve_finish (dx,
  // dz, ds). The affine solve's forward elimination runs inside factor_chain<true> instead, with
  // each block's inverse still in registers (solve_chain<true> then only substitutes back).
  template <int kMode>
  __device__ void solve(double smu, bool rx = false, bool step0 = true) {
    solve_rhs<kMode>(smu, rx);
    solve_chain<false>();
    solve_finish<false, false, true>(step0);
  }

  // One step of iterative refinement of the combined direction d = (dx, ds, dz, dy) against the
  // full KKT of sparse_pdipm_solver.py:412-439. The chains' explicit 12x12 block inverses are not
  // backward-stable along the stiff directions of S (the yaw-moment columns enter S_ii with
  // 1/(R + beta) = 1e4, and the packed store keeps one of the two rounding-different halves of each
  // symmetric inverse), so dy is off by ~eps cond |dy| and dx_u = Phi_u^-1 (r - N^T dy) multiplies
  // that by 1e4: 1e-7 relative in x after one iteration against the oracle's sparse LDL^T; and as
  // the barrier sharpens (W = z / s -> 1e8) the reduced foot rows r~ = -r_x - G^T D^-1 (r2 - W r3)
  // cancel against Phi_f dx_f. At degenerate iterates (s and z both at their 1e-8 clamps, Lambda
  // ~ 4e7, cond Phi_f ~ 4e12) rows 2 and 3 -- which ds, dz are formed from -- lose digits too: a
  // correction from rows 1 and 4 alone then stalls at ~1e-6 in dx while one from all four rows
  // reaches ~1e-11 (CPU emulation of this elimination, scripts/dual_refine_emu_stress.py;
  // profiles/r02/refinement_4row.txt). The correction K c = e of all four residuals,
  //   e1 = -r_x - (H + beta) dx - G^T dz - A^T dy   (foot columns: the other columns' Phi is
  //        diagonal with no G, so their row-1 residual is rounding only)
  //   e2 = r2 - (W ds + dz),   e3 = -r_s - (G dx + ds - delta dz),   e4 = -r_e - (A dx - delta dy)
  // is taken through the same elimination, block Gauss-Seidel:
  //   0. q = D^-1 (e2 - W e3) per inequality row; VV += q and r_s -= e3, so that solve_finish<true>'s
  //      re-formation dz = VV + Lambda G dx, ds = -r_s - G dx + delta dz yields dz + c_z, ds + c_s;
  //   1. dx_f += Phi_f^-1 (e1 - G^T q) on the foot columns (G^T (dz + q) in one pass over Z);
  //   2. rho = A_dyn dx + r_e - delta dy = A t_c - e4 (the x-moment rows are eliminated exactly by
  //      their 2x2 blocks);
  //   3. one more chain solve S c = rho; dy += c, dx -= Phi~^-1 A^T c (solve_finish<true>, which
  //      leaves row 1 as step 1 made it) and dz, ds re-formed from dx.
  // On the SURVEY workloads this sits at the dense-LU-vs-oracle floor over 512 envs per case at
  // K = 1/10/20 (profiles/r02/refinement_variants.txt). dy is parked in RXu (r_x's u part is dead
  // once step 1 has read it) while QV carries rho and then c.
  template <int t, bool kPark>
  __device__ void rho_slot(const double* TV, const double* Mc, const double* Pd, const double* Nd, double* QV,
                           double* DYs) {
    const ERow q = erow(fresh_lane(), t);
    const double v = arow<t>(TV, Mc, Pd, Nd, q);
    const int e = sink(q.valid, q.e, Lo::QV);
    const double dy = QV[e];  // read and rewritten by its owner lane only
    if (kPark) DYs[sink(q.valid, q.e, Lo::RXu)] = dy;
    QV[e] = (v + re[t]) - kDelta * dy;
  }
  // kAff: the affine (predictor) direction at a degenerate iterate (see the main loop): r_s stays
  // (the combined solve needs it), e3 goes to Z for solve_finish<true, true>, and dy is not parked
  // (RXu still feeds the combined solve)
  // row1 = false (refinement policy 3): the dual rows only -- no KKT row-1 foot correction
  template <bool kAff = false>
  SRBD_PHASE_ATTR __device__ void refine_rhs(bool row1 = true) {
    const int lane = fresh_lane();
    const double *Mc = at(Lo::Mc), *Nd = at(Lo::Nd), *Pd = at(Lo::Pd), *Gf = at(Lo::Gf), *Hu = at(Lo::Hu);
    double *TV = at(Lo::TV), *QV = at(Lo::QV), *DYs = at(Lo::RXu), *Zd = at(Lo::Z);
    if constexpr (kAff) {  // step 0 for the affine direction (the combined one ran it in its finish)
      double *VV = at(Lo::VV);
#pragma unroll
      for (int t = 0; t < SI; ++t) {
        const int q = lane + TPB * t;
        e3r[t] = 0.0;
        if (RegCtx<N>::full_slot(t, m) || q < m) {
          const int i = q >> 4, k = q & 15;
          const double gd = grow4(Gf, k, TV + nx + m24(i, 12));
          const double e3 = -rs[t] - ((gd + ds[t]) - kDelta * dz[t]);
          const double e2 = Zd[q] - (wd[t] * ds[t] + dz[t]);  // r2 parked in Z by solve_rhs
          const double qc = di[t] * (e2 - wd[t] * e3);
          VV[q] = VV[q] + qc;
          e3r[t] = e3;
          Zd[q] = dz[t] + qc;
        }
      }
    }
    qp_sync<TPB>();  // (the combined direction's step 0 ran in its solve_finish, kStep0 = 1)
    const int fl = lane;
    if (row1 && (unsigned)fl < 2u * N) {  // KKT row 1 on the foot columns: dx_f += Phi_f^-1 e1_f
      const int i = fl >> 1, f = fl & 1, b = 12 * i;
      const double* zf = Zd + 16 * i + 8 * f;
      const double* RXu = DYs;
      const double* g = Gf + g_row(8 * f);  // (G^T dz)_a over column a's structural rows (as solve_rhs)
      double gt[4];
      {
        double zk[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) zk[k] = zf[k];
        gt[0] = g[0] * zk[0] + g[4] * zk[1];
        gt[1] = g[9] * zk[2] + g[13] * zk[3];
        gt[3] = g[19] * zk[4] + g[23] * zk[5];
        double gz0 = 0.0, gz1 = 0.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          gz0 += g[4 * k + 2] * zk[k];
          gz1 += g[4 * (k + 4) + 2] * zk[k + 4];
        }
        gt[2] = gz0 + gz1;
      }
      double e1[4], c[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int j = foot_colj(f, a);
        const double ay = a < 3 ? ncol(Nd, j, QV + b, a) : ncol<false>(Nd, j, QV + b, 0);
        e1[a] = ((-RXu[b + j] - (Hu[j] + kBeta) * TV[nx + b + j]) - gt[a]) - ay;
      }
      phi_solve(fl, e1, c);
#pragma unroll
      for (int a = 0; a < 4; ++a) TV[nx + b + foot_colj(f, a)] += c[a];
    }
    qp_sync<TPB>();
    if (kAff) {  // Z is dead from here on: it keeps e3 for solve_finish<true, true>
#pragma unroll
      for (int t = 0; t < SI; ++t)
        if (full_slot(t, m) || lane + TPB * t < m) Zd[lane + TPB * t] = e3r[t];
    }
    rho_slot<0, !kAff>(TV, Mc, Pd, Nd, QV, DYs);
    rho_slot<1, !kAff>(TV, Mc, Pd, Nd, QV, DYs);
    qp_sync<TPB>();
    PROF_ADD(6);
  }

  // rx (combined solve only): recompute the x / scalar columns of t -- the affine direction was
  // refined, so its full finish overwrote them in TV
  template <int kMode>
  SRBD_PHASE_ATTR __device__ void solve_rhs(double smu, bool rx = false) {
    const int lane = fresh_lane();
    double *VV = at(Lo::VV), *TV = at(Lo::TV), *QV = at(Lo::QV), *Zr2 = at(Lo::Z);
    const double *RXu = at(Lo::RXu), *REm = at(Lo::REm), *IX = at(Lo::IX), *Gf = at(Lo::Gf),
                 *SG = at(Lo::SG), *Mc = at(Lo::Mc), *Nd = at(Lo::Nd), *Pd = at(Lo::Pd);
#pragma unroll
    for (int t = 0; t < SI; ++t) {
      const int q = lane + TPB * t;
      if (RegCtx<N>::full_slot(t, m) || q < m) {
        const double si = rcp3(s[t]);
        double r2 = -(si * (s[t] * z[t]));
        if (kMode == 1) r2 = r2 + -(si * (s[t] * z[t] + ds[t] * dz[t] - smu));
        Zr2[q] = r2;  // row 2's right-hand side for refine_rhs (Z is dead until the update)
        VV[q] = di[t] * (r2 + wd[t] * rs[t]);
      }
    }
    // The x columns and the scalar u columns of t = Phi^-1 r1~ do not depend on the complementarity
    // right-hand side, and the affine solve_finish (kAffine) leaves them in TV: the combined solve
    // (kMode 1) recomputes only the foot columns.
#pragma unroll
    for (int t = 0; t < SX; ++t) {
      const int c = lane + TPB * t;
      if ((kMode == 0 || rx) && (full_slot(t, nx) || c < nx)) TV[c] = -rxx[t] * IX[c - m24(div12(c), 12)];
    }
    qp_sync<TPB>();
    rhs_tasks<kMode>(lane, rx);
    qp_sync<TPB>();
    g_slot<0>(TV, Mc, Pd, Nd, QV);  // g = A_dyn t + r_e (dynamics rows, owner of r_e)
    g_slot<1>(TV, Mc, Pd, Nd, QV);
    qp_sync<TPB>();
    PROF_ADD(3);
  }

  // solve_rhs's per-stage tasks fl = lane: t = Phi^-1 r1~ on the foot columns (fl < 2 N),
  // r1~ = -r_x - G^T VV (G only on the foot columns, each foot through its 8 rows), and the scalar u
  // columns of t (2 N <= fl < 3 N, affine solve or rx only)
  template <int kMode>
  __device__ void rhs_tasks(int fl, bool rx) {
    double* TV = at(Lo::TV);
    const double *VV = at(Lo::VV), *RXu = at(Lo::RXu), *REm = at(Lo::REm), *Gf = at(Lo::Gf), *SG = at(Lo::SG);
    if ((unsigned)fl < (unsigned)(((kMode == 0 || rx) ? 3 : 2) * N)) {
      if (fl < 2 * N) {
        const int i = fl >> 1, f = fl & 1, b = 12 * i;
        double rv[4], tv[4];
        {
          const double* vv = VV + 16 * i + 8 * f;
          const double* g = Gf + g_row(8 * f);  // (G^T vv)_a over column a's structural rows
          double vk[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) vk[k] = vv[k];
          const double gfx = g[0] * vk[0] + g[4] * vk[1];
          const double gfy = g[9] * vk[2] + g[13] * vk[3];
          const double gmy = g[19] * vk[4] + g[23] * vk[5];
          double gz0 = 0.0, gz1 = 0.0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            gz0 += g[4 * k + 2] * vk[k];
            gz1 += g[4 * (k + 4) + 2] * vk[k + 4];
          }
          rv[0] = -RXu[b + foot_colj(f, 0)] - gfx;
          rv[1] = -RXu[b + foot_colj(f, 1)] - gfy;
          rv[2] = -RXu[b + foot_colj(f, 2)] - (gz0 + gz1);
          rv[3] = -RXu[b + foot_colj(f, 3)] - gmy;
        }
        phi_solve(fl, rv, tv);
#pragma unroll
        for (int a = 0; a < 4; ++a) TV[nx + b + foot_colj(f, a)] = tv[a];
      } else {
        const int i = fl - 2 * N, b = 12 * i;
        const double r4a = -REm[2 * i], r4b = -REm[2 * i + 1];
        TV[nx + b + 6] = (kDelta * -RXu[b + 6] + SG[6] * r4a) * SG[8];  // SG[8] = 1 / (phi6 delta + e6^2)
        TV[nx + b + 9] = (kDelta * -RXu[b + 9] + SG[7] * r4b) * SG[9];
        TV[nx + b + 8] = -RXu[b + 8] * SG[1];
        TV[nx + b + 11] = -RXu[b + 11] * SG[3];
      }
    }
  }

  // Twisted block solve (pdipm_srbd.hpp FastCtx::solve), w / v in registers. kBackOnly: the
  // forward elimination already ran in factor_chain<true>, which left w of every step in QV.
  template <bool kBackOnly>
  SRBD_PHASE_ATTR __device__ void solve_chain() {
    const int lane = fresh_lane();
    double* QV = at(Lo::QV);
    const double* DV = at(Lo::DV);
    if (lane < 32) {
      const int g = lane >> 4, l16 = lane & 15;
      const int r = l16 < 12 ? l16 : 11;
      const bool own = l16 < 12;
      const int pr = g ? perm12(r) : r;
      const int cnt = g ? nb : nf;
      const double* cc = at(Lo::Cc) + 24 * g;
      CoupleRow Cr, Ct;  // row r of Cg and of Cg^T (compact layout, see the header)
      uint32_t offs[12];
      load_chain_offs(lane, offs);
      {  // coefficients loaded from clamped indices and selected (no conditional loads)
        const bool ra = r < 3, rb = r >= 3 && r < 6, ta = r >= 6 && r < 9, tb = r >= 9;
        const int r3 = ra ? r : 0, r6 = rb ? r : 3, t6 = ta ? r : 6, t9 = tb ? r : 9;
        const double la0 = cc[12 + 3 * r3], la1 = cc[13 + 3 * r3], la2 = cc[14 + 3 * r3], lb = cc[21 + r6 - 3];
        const double ka0 = cc[12 + t6 - 6], ka1 = cc[15 + t6 - 6], ka2 = cc[18 + t6 - 6], kb = cc[12 + t9];
        Cr.d = cc[r];
        Cr.b = rb ? lb : 0.0;
        Cr.a0 = ra ? la0 : 0.0;
        Cr.a1 = ra ? la1 : 0.0;
        Cr.a2 = ra ? la2 : 0.0;
        Ct.d = Cr.d;
        Ct.b = tb ? kb : 0.0;
        Ct.a0 = ta ? ka0 : 0.0;
        Ct.a1 = ta ? ka1 : 0.0;
        Ct.a2 = ta ? ka2 : 0.0;
      }
      double w = 0.0, wv[T + 1];  // w / v per elimination step, indexed through selects
#pragma unroll
      for (int k = 0; k <= T; ++k) wv[k] = 0.0;
      if constexpr (kBackOnly) {  // w of every step from QV (stage i, element pr), mid included
#pragma unroll
        for (int t = 0; t < T; ++t)
          if (t < cnt) wv[t] = QV[12 * (g ? N - 1 - t : t) + pr];
        w = QV[12 * mid + pr];
      }
#pragma unroll
      for (int t = 0; t <= (kBackOnly ? -1 : T); ++t) {
        const bool mstep = (t == T);
        const int i = mstep ? mid : (g ? N - 1 - t : t);
        const bool act = mstep ? true : (t < cnt);
        const bool prev = mstep ? (cnt >= 1) : (t >= 1);
        const double q = fwd_rhs(act, prev, mstep, g, r, Cr, w, QV + 12 * i + pr);
        if (act && !(mstep && g == 1)) {
          const int imm = mstep ? kDvBytes * (N - 1) : 2 * kDvBytes * t;
          double Dr[12];
#pragma unroll
          for (int k = 0; k < 12; ++k) Dr[k] = dv_at(DV, offs[k], imm);
          w = dot_bc12(Dr, q);
#pragma unroll
          for (int k = 0; k <= T; ++k) wv[k] = (k == t) ? w : wv[k];
        }
      }
      // outward substitution from y_mid (group 0's last w; group 1 fetches row pi(r) of it)
      double y = w;
      if constexpr (!kBackOnly) {
        const double ym = __shfl(w, perm12(r), 64);
        if (own && g == 0) QV[12 * mid + r] = w;
        y = g ? ym : w;
      }
      // step te walks back from each group's last elimination step: both groups' blocks of step te
      // sit at 1248 te, and w_te is register wv[te]
#pragma unroll
      for (int te = T - 1; te >= 0; --te) {
        if (te < cnt) {
          const int i = g ? N - 1 - te : te;
          double Dr[12];
#pragma unroll
          for (int k = 0; k < 12; ++k) Dr[k] = dv_at(DV, offs[k], 2 * kDvBytes * te);
          y = dot_bc12_sub(Dr, couple_cty2(Ct, y), wv[te]);  // w_te - D^-1 Cg^T y_prev
          if (own) QV[12 * i + pr] = y;
        }
      }
    }
    qp_sync<TPB>();
    PROF_ADD(4);
  }

  // kRefine: the refinement step -- TV holds dx and QV the dual correction c, so the same updates
  // give dx - Phi~^-1 A^T c; the x-moment duals move by their 2x2 formula's increment, and dz, ds are
  // re-formed from the refined dx (with the combined solve's VV, r_s).
  // kAffine: the affine (predictor) direction, of which only ds and dz are consumed (step lengths,
  // mu_aff and the corrector's ds o dz, sparse_pdipm_solver.py:484-490): G touches only the foot
  // columns, so dx is finished on those alone (no x columns, no scalar columns, no x-moment duals).
  // kStep0: refine_rhs's step 0 for the combined direction fused into the row loop, where dz, ds,
  // G dx and VV are at hand -- e2, e3, q = D^-1 (e2 - W e3); VV += q, Z = dz + q for G^T (dz + q),
  // r_s -= e3 (step0 false: skipped at run time -- an iteration whose combined direction the refinement
  // policy leaves unrefined or refines in the dual rows only)
  template <bool kRefine = false, bool kAffine = false, bool kStep0 = false>
  SRBD_PHASE_ATTR __device__ void solve_finish(bool step0 = true) {
    const int lane = fresh_lane();
    double *VV = at(Lo::VV), *TV = at(Lo::TV), *QV = at(Lo::QV), *DYm = at(Lo::DYm);
    const double *RXu = at(Lo::RXu), *REm = at(Lo::REm), *IX = at(Lo::IX), *Gf = at(Lo::Gf),
                 *SG = at(Lo::SG), *Mc = at(Lo::Mc), *Nd = at(Lo::Nd), *Pd = at(Lo::Pd);
#pragma unroll
    for (int t = 0; t < SX; ++t) {  // dx (x part) = t - phi_x^-1 A^T dy
      const int c = lane + TPB * t;
      if (!kAffine && (full_slot(t, nx) || c < nx)) {
        const int k = div12(c) + 1, j = c - m24(k - 1, 12);
        double aty = Pd[j] * QV[12 * (k - 1) + j];
        const double mq = mcol(Mc, j, QV + 12 * (k < N ? k : N - 1));  // k = N: unused
        aty = fma(k < N ? 1.0 : 0.0, mq, aty);
        TV[c] = TV[c] - aty * IX[j];
      }
    }
    const int fl = lane;
    if ((unsigned)fl < (unsigned)((kAffine ? 2 : 3) * N)) {
      const bool foot = kAffine || fl < 2 * N;
      const int i = foot ? (fl >> 1) : fl - 2 * N;
      const int b = nx + 12 * i;
      const double* yi = QV + 12 * i;
      if (foot) {
        const int f = fl & 1;
        double av[4], tv[4];
#pragma unroll
        for (int a = 0; a < 3; ++a) av[a] = ncol(Nd, foot_colj(f, a), yi, a);
        av[3] = ncol<false>(Nd, foot_colj(f, 3), yi, 0);
        phi_solve(fl, av, tv);
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const int o = b + foot_colj(f, a);
          TV[o] = TV[o] - tv[a];
        }
      } else {
        const double r4a = kRefine ? 0.0 : -REm[2 * i], r4b = kRefine ? 0.0 : -REm[2 * i + 1];
        const double a6 = ncol<false>(Nd, 6, yi, 0), a9 = ncol<false>(Nd, 9, yi, 0);
        const double a8 = ncol<false>(Nd, 8, yi, 0), a11 = ncol<false>(Nd, 11, yi, 0);
        TV[b + 6] -= SG[0] * a6;
        TV[b + 9] -= SG[2] * a9;
        TV[b + 8] -= SG[1] * a8;
        TV[b + 11] -= SG[3] * a11;
        if constexpr (kRefine) {  // dy_E = (e rho - phi r4) / (phi delta + e^2), rho = -r_x - a
          DYm[2 * i] -= (SG[6] * a6) * SG[8];
          DYm[2 * i + 1] -= (SG[7] * a9) * SG[9];
        } else {
          const double rho6 = -RXu[12 * i + 6] - a6, rho9 = -RXu[12 * i + 9] - a9;
          DYm[2 * i] = (SG[6] * rho6 - SG[4] * r4a) * SG[8];
          DYm[2 * i + 1] = (SG[7] * rho9 - SG[5] * r4b) * SG[9];
        }
      }
    }
    qp_sync<TPB>();
#pragma unroll
    for (int t = 0; t < SI; ++t) {  // dz, ds (owner regs)
      const int q = lane + TPB * t;
      if (RegCtx<N>::full_slot(t, m) || q < m) {
        const int i = q >> 4, k = q & 15;
        const double gd = grow4(Gf, k, TV + nx + m24(i, 12));
        const double vq = VV[q];
        dz[t] = vq + di[t] * wd[t] * gd;
        // the affine refinement keeps r_s and parks its row-3 residual e3 in Z (refine_rhs<true>)
        const double r3 = (kRefine && kAffine) ? at(Lo::Z)[q] - rs[t] : -rs[t];
        ds[t] = r3 - gd + kDelta * dz[t];
        if (kStep0 && step0) {
          double* Zd = at(Lo::Z);
          const double e3 = -rs[t] - ((gd + ds[t]) - kDelta * dz[t]);
          const double e2 = Zd[q] - (wd[t] * ds[t] + dz[t]);  // r2 parked in Z by solve_rhs
          const double qc = di[t] * (e2 - wd[t] * e3);
          VV[q] = vq + qc;
          rs[t] = rs[t] - e3;
          Zd[q] = dz[t] + qc;
        }
      }
    }
    PROF_ADD(3);
  }

  __device__ double step_length(const double (&v)[SI], const double (&dv)[SI]) {
    const int lane = fresh_lane();
    double mn = INFINITY;
#pragma unroll
    for (int t = 0; t < SI; ++t) {
      const int q = lane + TPB * t;
      if (RegCtx<N>::full_slot(t, m) || q < m) {
        const bool c = dv[t] < 0.0;
        const double a = -v[t] * rcp3(dv[t]);
        mn = fmin(mn, (c ? a : 0.0) + (!c ? 1.0 : 0.0));
      }
    }
    mn = block_min(mn);
    return fmax(fmin(1.0, 0.99 * mn), 1e-12);
  }
  __device__ double step_min(const double (&v)[SI], const double (&dv)[SI]) {
    const int lane = fresh_lane();
    double mn = INFINITY;
#pragma unroll
    for (int t = 0; t < SI; ++t) {
      const int q = lane + TPB * t;
      if (RegCtx<N>::full_slot(t, m) || q < m) {
        const bool c = dv[t] < 0.0;
        const double a = -v[t] * rcp3(dv[t]);
        mn = fmin(mn, (c ? a : 0.0) + (!c ? 1.0 : 0.0));
      }
    }
    return mn;
  }
  // The primal and dual step lengths: at one wave per QP their two min-reductions run as one
  // interleaved DPP tree (the same values as two step_length calls)
  __device__ void step_lengths(double& ap, double& ad) {
    if constexpr (TPB == 64) {
      double mp = step_min(s, ds), md = step_min(z, dz);
      wave_min2(mp, md);
      ap = fmax(fmin(1.0, 0.99 * mp), 1e-12);
      ad = fmax(fmin(1.0, 0.99 * md), 1e-12);
    } else {
      ap = step_length(s, ds);
      ad = step_length(z, dz);
    }
  }
};

// Arguments of the fused former + solver kernel (srbd_mpc_solve_fused): the 17 qp_former inputs
// in, the QP's vectors f, b, d written once (row per env, re-read by the same lanes every Newton
// iteration; the matrices H, A, G never leave the kernel), the solver outputs out.
// The controller step (srbd_mpc_step) adds the input preparation in front (prep: the 17 former
// inputs are computed into LDS instead of read from memory) and the foot wrench / stance torque
// behind (wrench != null). Every out / vec pointer may be null: that array is not written.
struct FusedArgs {
  const double* in[17];
  double* vec[3];  // f (B, 24N), b (B, 14N), d (B, 16N), or null
  double* out[6];  // x, s, z, y, residuals(4), mu(1), each or null
  int N, n_iter, batch;
  double y0;
  int ctrl;        // 1: former inputs from prepare_env (prep) instead of in[]
  PrepArgs prep;
  float* wrench;   // (B, 2, 6) float32, or null
  const float *jac, *contact;  // (B, 2, 6, ndof), (B, 2) float32 for tau
  float* tau;      // (B, 2, ndof) float32, or null
  int ndof;
  int* status;     // (B) per-problem status word (pdipm.hpp kStatus*), or null
  int refine_policy;  // srbd_set_refinement_policy's word (include/srbd_mpc.h SRBD_REFINE_*)
  double refine_w;    // the W = z / s vote's threshold (INFINITY: no W vote)
};

// Body shared by the solver kernel (kFused = false: the QP comes from qp_former's CCS outputs and is
// checked for stage invariance) and the fused kernel (kFused = true: the stage blocks are computed
// here from the former inputs with qp_former's own device code, invariant by construction).
template <int N, bool kFused>
__device__ __forceinline__ void reg_kernel_body(const SolverArgs& args, const FusedArgs& fa) {
  using Lo = RegLayout<N>;
  constexpr int TPB = reg_tpb(N);
  // Static LDS sized by the horizon's layout (launched with 0 dynamic bytes): the addresses are
  // compile-time constants that fold into the instructions (a dynamic-LDS base is a link-time symbol
  // the backend re-adds as a literal 0 in every address computation: 118 v_add_u32 per kernel at N = 10)
  __shared__ __attribute__((aligned(16))) double smem[Lo::total];
  const int env = xcd_item(blockIdx.x, gridDim.x);
  if (env >= (kFused ? fa.batch : args.batch)) return;
  const int lane = threadIdx.x;
  constexpr int nz = Lo::nz, m = Lo::m, p = Lo::p, nx = Lo::nx, SI = Lo::SI;
  RegCtx<N, kFused> C;
  C.L = smem;
  C.lane = lane;
  double *Mc = smem + Lo::Mc, *Cc = smem + Lo::Cc, *Nd = smem + Lo::Nd, *Gf = smem + Lo::Gf,
         *K0 = smem + Lo::K0, *K1 = smem + Lo::K1, *Pd = smem + Lo::Pd, *IX = smem + Lo::IX,
         *Hu = smem + Lo::Hu, *SG = smem + Lo::SG;
  double* Md = smem + Lo::X;  // dense M while the constants are built (X is set at the iterate init)
  double e6 = 0.0, e9 = 0.0;  // x-moment coefficients (lane 0)

  if constexpr (kFused) {
    // ---- the stage blocks from the former inputs (qp_former.hpp's former_model) ----
    FormerLds& F = *reinterpret_cast<FormerLds*>(smem + Lo::TV);  // TV..DYm are free until the solve
    static_assert(sizeof(FormerLds) <= sizeof(double) * (Lo::total - Lo::TV), "former scratch fits");
    // The 17 former inputs of this env live in DV (dead until the first factor) for the whole
    // prologue: prepared there (controller step) or staged there from memory in one round trip
    static_assert(4 * 12 * N + 2 * N + 44 <= 80 * N, "former inputs fit the DV blocks");
    const double* P[17];
    double* o[17];
    {
      int off = 0;
#pragma unroll
      for (int i = 0; i < 17; ++i) {
        o[i] = smem + Lo::DV + off;
        P[i] = o[i];
        off += former_in_nnz(i, N);
      }
    }
    if (fa.ctrl) {  // controller step: the inputs are prepared here
      if (lane < 64) prepare_env(fa.prep, env, lane, o);
      qp_sync<TPB>();
      if (fa.prep.out[0]) {  // the caller also wants the prepared inputs in memory
#pragma unroll
        for (int i = 0; i < 17; ++i) {
          const int w = former_in_nnz(i, N);
          double* g = fa.prep.out[i] + (size_t)env * w;
          for (int e = lane; e < w; e += TPB) g[e] = o[i][e];
        }
      }
    } else {  // every load issued before any store: one memory round trip instead of the former
              // model's chain of dependent global reads (measured 60k cycles of prologue per QP)
      static_assert(12 * N <= 2 * TPB, "every former input row fits two passes of the QP's threads");
      double v[17][2];
#pragma unroll
      for (int i = 0; i < 17; ++i) {
        const int w = former_in_nnz(i, N);
        const double* g = fa.in[i] + (size_t)env * w;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int e = lane + TPB * t;
          v[i][t] = (TPB * t < w && e < w) ? g[e] : 0.0;
        }
      }
#pragma unroll
      for (int i = 0; i < 17; ++i) {
        const int w = former_in_nnz(i, N);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int e = lane + TPB * t;
          if (TPB * t < w && e < w) o[i][e] = v[i][t];
        }
      }
      qp_sync<TPB>();
    }
    former_model(F, P, lane);
    const double mu = P[6][0];
    for (int e = lane; e < 144; e += TPB) {
      const int r = e / 12, j = e % 12;
      const int om = c_tab.Mi[r][j], on = c_tab.Ni[r][j];
      Md[e] = (N >= 2 && om >= 0) ? F.XB[om] : 0.0;
      Nd[nd_idx(r, j)] = on >= 0 ? F.UB[on] : 0.0;
    }
    for (int e = lane; e < kGfSize; e += TPB) Gf[e] = 0.0;  // 16 rows x 4 (+ the foot-1 pad)
    if (lane < 12) {
      Pd[lane] = F.XB[c_tab.cpx[lane]];
      Hu[lane] = P[14][lane];       // H = diag(Q.., R..): u part R
      Hu[12 + lane] = P[13][lane];  // x part Q
    }
    if (lane == 0) {
      e6 = F.UB[c_tab.e6];
      e9 = F.UB[c_tab.e9];
    }
    qp_sync<TPB>();
    if (lane < 28) Gf[g_row(c_tab.grow[lane]) + foot_pos(c_tab.gcol[lane])] = former_g(lane, mu);
    // f, b, h straight into the registers of the lanes that use them (load_qp_vectors' mapping);
    // the rows reach memory only if the caller asked for them
#pragma unroll
    for (int t = 0; t < Lo::SX; ++t) {
      const int c = min(lane + TPB * t, nx - 1);
      C.fxr[t] = former_f(c, N, P[13], P[14], P[1], P[2], P[3]);
      C.fur[t] = former_f(nx + c, N, P[13], P[14], P[1], P[2], P[3]);
    }
#pragma unroll
    for (int t = 0; t < Lo::SE; ++t) {
      const auto q = RegCtx<N>::erow(lane, t);
      C.bvr[t] = former_b(q.valid ? q.e : 0, N, F);
    }
#pragma unroll
    for (int t = 0; t < SI; ++t) C.hvr[t] = former_d(min(lane + TPB * t, m - 1), N, P[2], P[12], mu);
    if (fa.vec[0]) {
      double* fw = fa.vec[0] + (size_t)env * nz;
#pragma unroll
      for (int t = 0; t < Lo::SX; ++t)
        if (lane + TPB * t < nx) {
          fw[lane + TPB * t] = C.fxr[t];
          fw[nx + lane + TPB * t] = C.fur[t];
        }
    }
    if (fa.vec[1]) {
      double* bw = fa.vec[1] + (size_t)env * p;
#pragma unroll
      for (int t = 0; t < Lo::SE; ++t) {
        const auto q = RegCtx<N>::erow(lane, t);
        if (q.valid) bw[q.e] = C.bvr[t];
      }
    }
    if (fa.vec[2]) {
      double* dw = fa.vec[2] + (size_t)env * m;
#pragma unroll
      for (int t = 0; t < SI; ++t)
        if (lane + TPB * t < m) dw[lane + TPB * t] = C.hvr[t];
    }
  } else {
    const int nA = nnz_A(N), nG = 28 * N;
    const double* Hg = solver_in(args, 0) + (size_t)env * nz;
    const double* Gg = solver_in(args, 1) + (size_t)env * nG;
    const double* Ag = solver_in(args, 2) + (size_t)env * nA;
    C.env_ = env;
    if constexpr (!RegCtx<N, kFused>::kArgRows) {
      C.fp_ = solver_in(args, 3) + (size_t)env * nz;
      C.hp_ = solver_in(args, 4) + (size_t)env * m;
      C.bp_ = solver_in(args, 5) + (size_t)env * p;
    }
    // ---- compact load (stage 0/1 slices) ----
    for (int e = lane; e < 144; e += TPB) {
      const int r = e / 12, j = e % 12;
      const int om = c_tab.Mi[r][j], on = c_tab.Ni[r][j];
      Md[e] = (N >= 2 && om >= 0) ? Ag[a_xblock(1) + om] : 0.0;
      Nd[nd_idx(r, j)] = on >= 0 ? Ag[a_ublock(N, 0) + on] : 0.0;
    }
    for (int e = lane; e < kGfSize; e += TPB) Gf[e] = 0.0;  // 16 rows x 4 (+ the foot-1 pad)
    if (lane < 12) {
      Pd[lane] = Ag[a_pidx(c_tab, N, 0, lane)];
      Hu[lane] = Hg[nx + lane];
      Hu[12 + lane] = Hg[lane];
    }
    qp_sync<TPB>();
    if (lane < 28) Gf[g_row(c_tab.grow[lane]) + foot_pos(c_tab.gcol[lane])] = Gg[lane];
    // ---- stage-invariance check (bitwise): every periodic block equals the first one ----
    // x_k blocks (36 values, k = 1..N-1) vs x_1's; the x_N single entries vs x_1's +I entries (P);
    // u_i blocks (86 values) vs u_0's (the latter include the x-moment entries e6/e9)
    bool bad = false;
    for (int e = lane; e < nA; e += TPB) {
      int ref;
      if (e < 36 * (N - 1)) ref = e % 36;
      else if (e < a_ubase(N)) ref = c_tab.cpx[e - 36 * (N - 1)];
      else ref = a_ubase(N) + (e - a_ubase(N)) % 86;
      bad |= !(Ag[e] == Ag[ref]);
    }
    for (int e = lane; e < nG; e += TPB) bad |= !(Gg[e] == Gg[e % 28]);
    for (int e = lane; e < nz; e += TPB) bad |= !(Hg[e] == Hg[(e < nx ? 0 : nx) + e % 12]);
    bad = __any(bad);
    if constexpr (TPB > 64) {  // one verdict for the whole QP (all its waves leave or all stay)
      int* vr = reinterpret_cast<int*>(smem + Lo::RED);
      if ((lane & 63) == 0) vr[lane >> 6] = bad;
      qp_sync<TPB>();
      bool any = false;
#pragma unroll
      for (int w = 0; w < TPB / 64; ++w) any = any || vr[w];
      bad = any;
      qp_sync<TPB>();  // RED is reused by the first block reduction
    }
    if (bad) {  // not stage-invariant: the general solve, in this launch (pdipm_general_scratch)
      // the kernel's sole argument; the QP's LDS holds the slot hand-over and the chain arrays
      pdipm_general_scratch<N>(kernel_args(), env, smem, Lo::total);
      return;
    }
    // loaded only now: a value held across the fallback call would be saved around it (the callee
    // clobbers every VGPR), i.e. spill in the fast path too
    C.load_qp_vectors();
    if (lane == 0) {
      e6 = Ag[a_ubase(N) + c_tab.e6];
      e9 = Ag[a_ubase(N) + c_tab.e9];
    }
  }
  // ---- per-QP constants ----
  for (int l = lane; l < 78; l += TPB) reinterpret_cast<uint8_t*>(smem + Lo::TRI)[l] = c_tab.dvo[l];
  if (lane < 12) IX[lane] = 1.0 / (Hu[12 + lane] + kBeta);
  if (lane == 0) {
    const double p6 = Hu[6] + kBeta, p9 = Hu[9] + kBeta;
    SG[0] = kDelta / (p6 * kDelta + e6 * e6);
    SG[1] = 1.0 / (Hu[8] + kBeta);
    SG[2] = kDelta / (p9 * kDelta + e9 * e9);
    SG[3] = 1.0 / (Hu[11] + kBeta);
    SG[4] = p6;
    SG[5] = p9;
    SG[6] = e6;
    SG[7] = e9;
    SG[8] = 1.0 / (p6 * kDelta + e6 * e6);
    SG[9] = 1.0 / (p9 * kDelta + e9 * e9);
  }
  qp_sync<TPB>();
  if (lane < 24) {  // compact M and C (C = M diag(P / phi_x)); group 1's block is pi C^T pi^T
    int r, j;
    if (lane < 12) { r = lane; j = lane; }
    else if (lane < 21) { r = (lane - 12) / 3; j = 6 + (lane - 12) % 3; }
    else { r = lane - 21 + 3; j = r + 6; }
    const double mv = Md[r * 12 + j];
    Mc[lane] = mv;
    const double cv = mv * (Pd[j] * IX[j]);
    Cc[lane] = cv;
    // pi C^T pi^T: diag c <- C[pi c][pi c]; a-part (c, 6+k) <- C[k][c+6]; b-part unchanged
    int l1;
    if (lane < 12) l1 = perm12c(lane);
    else if (lane < 21) l1 = 12 + 3 * (j - 6) + r;  // entry (r, 6 + k) lands at (k, 6 + r)
    else l1 = lane;
    Cc[24 + l1] = cv;
  }
  for (int e = lane; e < 78; e += TPB) {
    int r, c;
    tri_rc(e, r, c);
    double k0 = (r == c) ? Pd[r] * Pd[r] * IX[r] + kDelta : 0.0;
    k0 += Nd[nd_idx(r, 6)] * Nd[nd_idx(c, 6)] * SG[0] + Nd[nd_idx(r, 8)] * Nd[nd_idx(c, 8)] * SG[1] +
          Nd[nd_idx(r, 9)] * Nd[nd_idx(c, 9)] * SG[2] + Nd[nd_idx(r, 11)] * Nd[nd_idx(c, 11)] * SG[3];
    double k1 = k0;
#pragma unroll
    for (int j = 0; j < 12; ++j) k1 += Md[r * 12 + j] * Md[c * 12 + j] * IX[j];
    K0[e] = k0;
    K1[e] = k1;
  }
  // ---- iterate ----
  // X aliases the dense M the K0 / K1 loop above reads: with two waves, the other wave must be past
  // that loop before X is written (one wave runs both loops in order)
  if constexpr (TPB > 64) qp_sync<TPB>();
  double *X = smem + Lo::X, *Z = smem + Lo::Z, *Y = smem + Lo::Y;
  if (!kFused && args.init_mode == 2) {  // _ccs cold start (sparse_pdipm_solver.py:30-35)
    const double* xg = solver_in(args, 6) + (size_t)env * nz;
    for (int e = lane; e < nz; e += TPB) X[e] = xg[e];
    qp_sync<TPB>();
#pragma unroll
    for (int t = 0; t < SI; ++t) {
      const int q = lane + TPB * t;
      if (RegCtx<N>::full_slot(t, m) || q < m) {
        C.s[t] = fmax(C.hval(t, q) - ccs_gx(solver_in(args, 1) + (size_t)env * 28 * N, q, X + nx), 1.0);
        C.z[t] = 1.0;
        Z[q] = 1.0;
      }
    }
    for (int e = lane; e < p; e += TPB) Y[e] = 0.0;
  } else if (!kFused && args.init_mode == 0) {
    const double* xg = solver_in(args, 6) + (size_t)env * nz;
    const double* sg = solver_in(args, 7) + (size_t)env * m;
    const double* zg = solver_in(args, 8) + (size_t)env * m;
    const double* yg = solver_in(args, 9) + (size_t)env * p;
    for (int e = lane; e < nz; e += TPB) X[e] = xg[e];
#pragma unroll
    for (int t = 0; t < SI; ++t) {
      const int q = lane + TPB * t;
      if (RegCtx<N>::full_slot(t, m) || q < m) {
        C.s[t] = sg[q];
        C.z[t] = zg[q];
        Z[q] = C.z[t];
      }
    }
    for (int e = lane; e < p; e += TPB) Y[e] = yg[e];
  } else {
    for (int e = lane; e < nz; e += TPB) X[e] = 0.0;
#pragma unroll
    for (int t = 0; t < SI; ++t) {
      const int q = lane + TPB * t;
      if (RegCtx<N>::full_slot(t, m) || q < m) {
        C.s[t] = fmax(C.hval(t, q) - 0.0, 1.0);
        C.z[t] = 1.0;
        Z[q] = 1.0;
      }
    }
    for (int e = lane; e < p; e += TPB) Y[e] = kFused ? fa.y0 : args.y0;
  }
  qp_sync<TPB>();

  double res0 = 0.0, res1 = 0.0, res2 = 0.0, mu_new = 0.0;
  const double* TV = smem + Lo::TV;
  const double* QV = smem + Lo::QV;
  const double* DYm = smem + Lo::DYm;
  const double* RXu = smem + Lo::RXu;
  PROF_MARK_CTX(C);
  const int n_iter = kFused ? fa.n_iter : args.n_iter;
  const int rpol = kFused ? fa.refine_policy : args.refine_policy;
  const double rw = kFused ? fa.refine_w : args.refine_w;
  for (int it = 0; it < n_iter; ++it) {
    if constexpr (TPB == 64 && SRBD_PROGRESS_PRIO) {
      // Wave priority falls with this QP's progress (3 over the first quarter of the iterations, 0
      // over the last): of the two waves sharing a SIMD the one further behind issues first, so
      // they finish together instead of the younger wave running its tail alone (the SIMD's
      // default is oldest-first). Not at N = 20, whose QPs span two waves joined by barriers.
      const int lvl = 3 - (4 * it) / n_iter;
      if (lvl >= 3) __builtin_amdgcn_s_setprio(3);
      else if (lvl == 2) __builtin_amdgcn_s_setprio(2);
      else if (lvl == 1) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    double mu = C.residuals(it == 0);
    if (it > 0) mu = mu_new;
    // An ill-conditioned iterate -- some row with W = z / s >= refine_w (1e4 in mode 0), e.g. an s
    // at or near its 1e-8 clamp (sparse_pdipm_solver.py:520) -- is where the reduced solve's affine
    // ds, dz lose digits; their error enters sigma and the corrector, and the trajectory drifts from the
    // reference's (profiles/r02/refinement_4row.txt; round 5: scripts/parity_fuzz.py found iterates at
    // W 4.5e3 .. 1.2e8 with s above the clamp drifting to 1e-4 in z, profiles/r05/parity_fuzz.txt).
    // Such iterations also refine the affine direction (the QP is one wave or joined ones: a uniform
    // branch); the bench workload has W >= 1e3 in ~4 % of its QP iterations (round 5's mode 0). The refinement policy
    // (srbd_set_refinement_policy, a kernel argument) adds iterations by position -- every one
    // (srbd_set_refinement(1), as the LDS-resident and general kernels always do), the first k, the last k --
    // and, in mode 0 since round 6, the iterate every solve starts from: all duals z at their initial 1 (the
    // GPU caller's and the _ccs init), where the cold start's Newton step is largest (round 5's mode 0 left 7 of
    // its 23 failing _ccs-campaign cases at K = 1 from there). A property of the iterate, not of the
    // iteration index, so 4 chained 5-iteration calls still equal one 20-iteration call bit for bit.
    bool degen;
    {
      const int l = C.fresh_lane();
      bool p = false, q = (rpol & kRefineAffineAtInit) != 0;
#pragma unroll
      for (int t = 0; t < SI; ++t)
        if (RegCtx<N>::full_slot(t, m) || l + TPB * t < m) {
          p = p || (C.s[t] <= 1e-8) || (C.z[t] >= rw * C.s[t]);
          q = q && (C.z[t] == 1.0);
        }
      degen = (rpol & kRefineAffineAll) || it < ((rpol >> 8) & 255) || it >= n_iter - ((rpol >> 16) & 255) ||
              C.block_any_or_all(p, q);
    }
    // the combined direction's refinement (SRBD_REFINE_COMBINED): every iteration in the product
    constexpr int cpol = SRBD_REFINE_COMBINED;
    const bool refc = cpol == 0 || cpol == 3 || (cpol == 2 && it >= n_iter / 2);
    int ul = C.fresh_lane();
    if (it == n_iter - 1) {  // residual norms of the last iteration (refine_rhs reuses r_x, r_e)
      double a = 0.0, b = 0.0, c = 0.0;
#pragma unroll
      for (int t = 0; t < Lo::SX; ++t)
        if (RegCtx<N>::full_slot(t, nx) || ul + TPB * t < nx) a += C.rxx[t] * C.rxx[t] + RXu[ul + TPB * t] * RXu[ul + TPB * t];
#pragma unroll
      for (int t = 0; t < SI; ++t)
        if (RegCtx<N>::full_slot(t, m) || ul + TPB * t < m) b += C.rs[t] * C.rs[t];
#pragma unroll
      for (int t = 0; t < Lo::SE; ++t)
        if (RegCtx<N>::erow(ul, t).valid) c += C.re[t] * C.re[t];
      res0 = sqrt(C.block_sum(a));
      res1 = sqrt(C.block_sum(b));
      res2 = sqrt(C.block_sum(c));
    }
    PROF_ADD_CTX(C, 0);
    C.factor_build();
    C.template solve_rhs<0>(0.0);
    C.template factor_chain<true>();  // + the affine forward elimination
    C.template solve_chain<true>();
    if (degen) {  // full affine finish (rho needs all of dx), then the 4-row refinement
      C.template solve_finish<false, false>();
      C.template refine_rhs<true>();
      C.template solve_chain<false>();
      C.template solve_finish<true, true>();
    } else {
      C.template solve_finish<false, true>();
    }
    double ap, ad;
    C.step_lengths(ap, ad);
    double sza = 0.0;
    ul = C.fresh_lane();
#pragma unroll
    for (int t = 0; t < SI; ++t)
      if (RegCtx<N>::full_slot(t, m) || ul + TPB * t < m) sza += (C.s[t] + ap * C.ds[t]) * (C.z[t] + ad * C.dz[t]);
    const double mu_aff = C.block_sum(sza) / m;
    const double ratio = mu_aff / mu;
    const double sigma = ratio * ratio * ratio;  // (mu_aff / mu)^3, sparse_pdipm_solver.py:487
    qp_sync<TPB>();
    PROF_ADD_CTX(C, 5);
    // (spelling the phases out here costs N = 20 spills)
    C.template solve<1>(sigma * mu * 1.0, degen, refc && cpol != 3);
    // one refinement step in EVERY iteration by default: in round 2 (explicit foot-block inverses)
    // refining only the last 1 or 3 iterations left the K = 10 / 20 parity where no refinement has it,
    // only the first 3 / 5 / 7 let the degenerate duals of K = 20 drift to 2e-5
    // (profiles/r02/refinement_parity.txt, refinement_variants.txt); round 6 re-measures
    if (refc) {
      C.refine_rhs(cpol != 3);
      C.template solve_chain<false>();
      C.template solve_finish<true>();
    }
    double apc, adc;
    C.step_lengths(apc, adc);
    // status bit 1 (a step length at its 1e-12 floor in the last iteration), kept in LDS: SG[15] is
    // unused (SG[0..9] are the x-moment constants) and a register held across the loop would spill
    if (it == n_iter - 1 && lane == 0) SG[15] = (apc <= 1e-12 || adc <= 1e-12) ? 1.0 : 0.0;
    qp_sync<TPB>();
    double szn = 0.0;
    ul = C.fresh_lane();
#pragma unroll
    for (int t = 0; t < (nz + TPB - 1) / TPB; ++t) {
      const int e = ul + TPB * t;
      if (RegCtx<N>::full_slot(t, nz) || e < nz) X[e] = X[e] + apc * TV[e];
    }
#pragma unroll
    for (int t = 0; t < SI; ++t) {
      const int q = ul + TPB * t;
      if (RegCtx<N>::full_slot(t, m) || q < m) {
        const double sn = fmax(C.s[t] + apc * C.ds[t], 1e-8);
        const double zn = fmax(fmax(C.z[t] + adc * C.dz[t], 1e-8), 1e-8);
        C.s[t] = sn;
        C.z[t] = zn;
        Z[q] = zn;
        szn += sn * zn;
      }
    }
    // dy = the combined solve's dy (parked in RXu by refine_rhs) + the refinement's correction (an
    // unrefined iteration: the combined solve's dy, in QV)
#pragma unroll
    for (int t = 0; t < (p + TPB - 1) / TPB; ++t) {
      const int e = ul + TPB * t;
      if (RegCtx<N>::full_slot(t, p) || e < p) {
        const double dye = e < nx ? (refc ? RXu[e] : 0.0) + QV[e] : DYm[e - nx];
        Y[e] = Y[e] + adc * dye;
      }
    }
    mu_new = C.block_sum(szn) / m;
    qp_sync<TPB>();
    PROF_ADD_CTX(C, 5);
  }
  PROF_FLUSH(C);
  auto outp = [&](int k) { return kFused ? fa.out[k] : solver_out(args, k); };
  if (double* xo = outp(0)) {
    xo += (size_t)env * nz;
    for (int e = lane; e < nz; e += TPB) xo[e] = X[e];
  }
  double* so = outp(1);
  double* zo = outp(2);
#pragma unroll
  for (int t = 0; t < SI; ++t) {
    const int q = lane + TPB * t;
    if (q < m) {
      if (so) so[(size_t)env * m + q] = C.s[t];
      if (zo) zo[(size_t)env * m + q] = C.z[t];
    }
  }
  if (double* yo = outp(3)) {
    yo += (size_t)env * p;
    for (int e = lane; e < p; e += TPB) yo[e] = Y[e];
  }
  if (lane == 0) {
    if (double* ro = outp(4)) {
      ro += (size_t)env * 4;
      ro[0] = res0;
      ro[1] = res1;
      ro[2] = res2;
      ro[3] = mu_new;
    }
    if (double* mo = outp(5)) mo[env] = mu_new;
  }
  if (int* st = kFused ? fa.status : args.status) {  // uniform: every wave takes part in the vote
    const int ul = C.fresh_lane();
    bool nf = ul == 0 && not_finite(mu_new);
    for (int e = ul; e < nz; e += TPB) nf = nf || not_finite(X[e]);
    for (int e = ul; e < p; e += TPB) nf = nf || not_finite(Y[e]);
#pragma unroll
    for (int t = 0; t < SI; ++t)
      if (RegCtx<N>::full_slot(t, m) || ul + TPB * t < m) nf = nf || not_finite(C.s[t]) || not_finite(C.z[t]);
    nf = C.block_any(nf);
    if (lane == 0) st[env] = (nf ? kStatusNonFinite : 0) | (SG[15] != 0.0 ? kStatusStepFloor : 0);
  }
  if constexpr (kFused) {
    if (fa.wrench) {  // u0 -> foot wrench (+ stance torque): srbd_u0_wrench_torque's arithmetic
      const float* Rm = fa.prep.rotation_body + 9 * (size_t)env;
      float* wl = reinterpret_cast<float*>(smem + Lo::TV);  // TV is dead after the last update
      if (lane < 12) {
        const float w = wrench_entry(X + nx, Rm, lane);
        fa.wrench[(size_t)env * 12 + lane] = w;
        wl[lane] = w;
      }
      if (fa.tau) {
        qp_sync<TPB>();
        const int nd = fa.ndof;
        for (int q = lane; q < 2 * nd; q += TPB) {
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
}

// Device code generation of the register kernels: no SILoadStoreOptimizer (the backend pass that
// pairs adjacent ds_read_b64 / ds_write_b64 into ds_read2_b64 / ds_write2_b64). A read2_b64 takes
// 8 LDS cycles (two accesses of 4 x 16 lanes, 32-bank mapping) where two ds_read_b64 take 4, and
// LDS is this kernel's busiest unit: without the pairing the fused N = 10 step runs 2.9 % faster
// (0.666 -> 0.646 ms; 12,955 -> 14,644 LDS instructions, 190k -> 184k wave cycles per QP;
// profiles/r03/no_ds_pairing.txt). Pairs the IR load-store vectorizer forms are kept.
#if defined(__HIP_DEVICE_COMPILE__)
#define SRBD_NO_DS_PAIRING __attribute__((target("no-load-store-opt")))
#else
#define SRBD_NO_DS_PAIRING
#endif

// at most 2 waves per SIMD (<= 256 registers): 2 one-wave QPs (N <= 10) per SIMD, or the waves of
// two-wave (N <= 21), three-wave (N <= 24) and four-wave (N <= 32) QPs
template <int N>
__global__ __launch_bounds__(reg_tpb(N), 2) SRBD_NO_DS_PAIRING void pdipm_srbd_reg_kernel(SolverArgs args) {
  reg_kernel_body<N, false>(args, FusedArgs{});
}

template <int N>
__global__ __launch_bounds__(reg_tpb(N), 2) SRBD_NO_DS_PAIRING void mpc_step_reg_kernel(FusedArgs fa) {
  reg_kernel_body<N, true>(SolverArgs{}, fa);
}

}  // namespace srbd
