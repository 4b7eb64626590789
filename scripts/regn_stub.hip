// regn_stub.hip -- diagnostic builds only (scripts/build_variant.py --no-regn): no register kernels at
// the horizons other than 10 and 20 (they then run the LDS-resident kernels), so a variant of the
// N = 10 / 20 kernels links in about a minute instead of the seven the srbd_regN.hip unit takes.
#define SRBD_NO_GENERAL_KERNEL
#include "../biped_pympc_amd/csrc/regN.hpp"

namespace srbd {
namespace regn {
bool supported(int) { return false; }
size_t lds_bytes(int) { return 0; }
const void* solver_kernel(int) { return nullptr; }
const void* step_kernel(int) { return nullptr; }
void launch_solver(int, const SolverArgs&, hipStream_t) {}
void launch_step(int, const FusedArgs&, hipStream_t) {}
}  // namespace regn
}  // namespace srbd
