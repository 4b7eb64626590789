// regN.hpp -- the register-resident kernels at the horizons other than 10 and 20 that they support
// (pdipm_srbd_reg.hpp reg_horizon: 2..32 except 10 and 20), compiled in their own translation unit
// (srbd_regN.hip, with the register-pressure trackers as the N = 20 unit) and dispatched by horizon
// at run time. Every other horizon runs the LDS-resident kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "pdipm_srbd.hpp"

namespace srbd {
struct FusedArgs;
namespace regn {
bool supported(int N);        // a register kernel instantiated here for this horizon
size_t lds_bytes(int N);      // RegLayout<N> in bytes
const void* solver_kernel(int N);
const void* step_kernel(int N);
// static LDS (RegLayout<N>): launched with 0 dynamic bytes
void launch_solver(int N, const SolverArgs& a, hipStream_t s);
void launch_step(int N, const FusedArgs& a, hipStream_t s);
}  // namespace regn
}  // namespace srbd
