// srbd_reg20.hip -- second translation unit of libsrbd_mpc.so: the N = 20 register-resident
// kernels (see reg20.hpp for why they are compiled apart). Launch geometry as in srbd_mpc.hip.
#define SRBD_NO_GENERAL_KERNEL
#include "reg20.hpp"

#include "pdipm_srbd_reg.hpp"

namespace srbd {
namespace reg20 {
const void* solver_kernel() { return (const void*)pdipm_srbd_reg_kernel<20>; }
const void* step_kernel() { return (const void*)mpc_step_reg_kernel<20>; }
void launch_solver(const SolverArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(pdipm_srbd_reg_kernel<20>, dim3(a.batch), dim3(reg_tpb(20)), 0, s, a);
}
void launch_step(const FusedArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(mpc_step_reg_kernel<20>, dim3(a.batch), dim3(reg_tpb(20)), 0, s, a);
}
}  // namespace reg20
}  // namespace srbd
