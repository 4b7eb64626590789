// phase_prof.hpp -- diagnostic phase stamps for the solver kernels (never part of the product build).
// Force-included by the diagnostic builds (hipcc -include scripts/phase_prof.hpp): the phase markers
// of csrc/srbd_common.hpp become s_memtime stamps; lane 0 of every wave accumulates per-phase
// shader-clock cycles into srbd_g_phase_cycles, read and reset by srbd_debug_phase_cycles().
#pragma once
#include <hip/hip_runtime.h>

__device__ unsigned long long srbd_g_phase_cycles[32];
#define PROF_DECL unsigned long long prof_t0_ = 0, prof_acc_[16] = {0};
#define PROF_MARK() (prof_t0_ = __builtin_amdgcn_s_memtime())
#define PROF_ADD(k)                                                  \
  do {                                                               \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();      \
    prof_acc_[k] += t_ - prof_t0_;                                   \
    prof_t0_ = t_;                                                   \
  } while (0)
// lane 0 of wave 0 into slots 0..15, lane 0 of wave 1 (two-wave QPs) into slots 16..31
#define PROF_FLUSH(ctx)                                              \
  if ((threadIdx.x & 63) == 0 && threadIdx.x < 128)                  \
    for (int k_ = 0; k_ < 16; ++k_)                                  \
      atomicAdd(&srbd_g_phase_cycles[16 * (threadIdx.x >> 6) + k_], (ctx).prof_acc_[k_]);
#define PROF_NOW() __builtin_amdgcn_s_memtime()
#define PROF_SPAN(k, t0) (prof_acc_[k] += __builtin_amdgcn_s_memtime() - (t0))
#define PROF_MARK_CTX(ctx) ((ctx).prof_t0_ = __builtin_amdgcn_s_memtime())
#define PROF_ADD_CTX(ctx, k)                                         \
  do {                                                               \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();      \
    (ctx).prof_acc_[k] += t_ - (ctx).prof_t0_;                       \
    (ctx).prof_t0_ = t_;                                             \
  } while (0)

// read and reset the per-phase cycle accumulators (32: wave 0, then wave 1)
extern "C" int srbd_debug_phase_cycles(unsigned long long* out16) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(srbd_g_phase_cycles), 32 * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  unsigned long long z[32] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(srbd_g_phase_cycles), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
