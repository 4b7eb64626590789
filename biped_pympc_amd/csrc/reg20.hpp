// reg20.hpp -- the N = 20 register-resident kernels, compiled in their own translation unit
// (srbd_reg20.hip) so that it can use the AMDGPU register-pressure trackers in the scheduler
// (-mllvm -amdgpu-use-amdgpu-trackers=1): they remove the 10 VGPRs the N = 20 kernel otherwise
// spills (fused step -1.3 %), while the same flag costs the N = 10 kernel +0.5 %
// (profiles/r01/sched_variants.txt). Without SRBD_SPLIT_REG20 the main unit instantiates them.
#pragma once
#include <hip/hip_runtime.h>

#include "pdipm_srbd.hpp"

namespace srbd {
struct FusedArgs;
namespace reg20 {
const void* solver_kernel();  // pdipm_srbd_reg_kernel<20>
const void* step_kernel();    // mpc_step_reg_kernel<20>
void launch_solver(const SolverArgs& a, hipStream_t s);
void launch_step(const FusedArgs& a, hipStream_t s);
}  // namespace reg20
}  // namespace srbd
