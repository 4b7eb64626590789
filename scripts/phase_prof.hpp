// phase_prof.hpp -- diagnostic phase stamps for the solver kernels (never part of the product build).
// Force-included by the diagnostic builds (hipcc -include scripts/phase_prof.hpp): the phase markers
// of csrc/srbd_common.hpp become s_memtime stamps; lane 0 of every wave accumulates per-phase
// shader-clock cycles into srbd_g_phase_cycles, read and reset by srbd_debug_phase_cycles().
#pragma once
#include <hip/hip_runtime.h>

__device__ unsigned long long srbd_g_phase_cycles[16];
#define PROF_DECL unsigned long long prof_t0_ = 0, prof_acc_[16] = {0};
#define PROF_MARK() (prof_t0_ = __builtin_amdgcn_s_memtime())
#define PROF_ADD(k)                                                  \
  do {                                                               \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();      \
    prof_acc_[k] += t_ - prof_t0_;                                   \
    prof_t0_ = t_;                                                   \
  } while (0)
#define PROF_FLUSH(ctx)                                              \
  if (threadIdx.x == 0)                                              \
    for (int k_ = 0; k_ < 16; ++k_) atomicAdd(&srbd_g_phase_cycles[k_], (ctx).prof_acc_[k_]);
#define PROF_MARK_CTX(ctx) ((ctx).prof_t0_ = __builtin_amdgcn_s_memtime())
#define PROF_ADD_CTX(ctx, k)                                         \
  do {                                                               \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();      \
    (ctx).prof_acc_[k] += t_ - (ctx).prof_t0_;                       \
    (ctx).prof_t0_ = t_;                                             \
  } while (0)

// read and reset the per-phase cycle accumulators
extern "C" int srbd_debug_phase_cycles(unsigned long long* out16) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(srbd_g_phase_cycles), 16 * sizeof(unsigned long long)) != hipSuccess)
    return -1;
  unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(srbd_g_phase_cycles), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
