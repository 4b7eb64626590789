// srbd_regN.hip -- third translation unit of libsrbd_mpc.so: the register-resident solver and
// fused-step kernels at N = 2..32 except 10 and 20 (regN.hpp). Launch geometry as in srbd_mpc.hip.
#define SRBD_NO_GENERAL_KERNEL
#include "regN.hpp"

#include "pdipm_srbd_reg.hpp"

namespace srbd {
namespace regn {

// The horizons in six parts of about equal compile time; SRBD_REGN_PART = k (0..5) instantiates
// part k only -- for the ISA audit (tests/test_isa_hazards.py), which compiles the parts in parallel.
// The product build defines no part: every horizon.
#define SRBD_REGN_P0(X) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(11) X(12) X(13)
#define SRBD_REGN_P1(X) X(14) X(15) X(16) X(17) X(18)
#define SRBD_REGN_P2(X) X(19) X(21) X(22) X(23)
#define SRBD_REGN_P3(X) X(24) X(25) X(26)
#define SRBD_REGN_P4(X) X(27) X(28) X(29)
#define SRBD_REGN_P5(X) X(30) X(31) X(32)
#if !defined(SRBD_REGN_PART)
#define SRBD_REGN_HORIZONS(X) \
  SRBD_REGN_P0(X) SRBD_REGN_P1(X) SRBD_REGN_P2(X) SRBD_REGN_P3(X) SRBD_REGN_P4(X) SRBD_REGN_P5(X)
#elif SRBD_REGN_PART == 0
#define SRBD_REGN_HORIZONS(X) SRBD_REGN_P0(X)
#elif SRBD_REGN_PART == 1
#define SRBD_REGN_HORIZONS(X) SRBD_REGN_P1(X)
#elif SRBD_REGN_PART == 2
#define SRBD_REGN_HORIZONS(X) SRBD_REGN_P2(X)
#elif SRBD_REGN_PART == 3
#define SRBD_REGN_HORIZONS(X) SRBD_REGN_P3(X)
#elif SRBD_REGN_PART == 4
#define SRBD_REGN_HORIZONS(X) SRBD_REGN_P4(X)
#else
#define SRBD_REGN_HORIZONS(X) SRBD_REGN_P5(X)
#endif

bool supported(int N) {
  switch (N) {
#define SRBD_CASE(n) case n: return true;
    SRBD_REGN_HORIZONS(SRBD_CASE)
#undef SRBD_CASE
    default: return false;
  }
}

size_t lds_bytes(int N) {
  switch (N) {
#define SRBD_CASE(n) case n: return sizeof(double) * (size_t)RegLayout<n>::total;
    SRBD_REGN_HORIZONS(SRBD_CASE)
#undef SRBD_CASE
    default: return 0;
  }
}

const void* solver_kernel(int N) {
  switch (N) {
#define SRBD_CASE(n) case n: return (const void*)pdipm_srbd_reg_kernel<n>;
    SRBD_REGN_HORIZONS(SRBD_CASE)
#undef SRBD_CASE
    default: return nullptr;
  }
}

const void* step_kernel(int N) {
  switch (N) {
#define SRBD_CASE(n) case n: return (const void*)mpc_step_reg_kernel<n>;
    SRBD_REGN_HORIZONS(SRBD_CASE)
#undef SRBD_CASE
    default: return nullptr;
  }
}

void launch_solver(int N, const SolverArgs& a, hipStream_t s) {
  switch (N) {
#define SRBD_CASE(n) \
  case n: hipLaunchKernelGGL(pdipm_srbd_reg_kernel<n>, dim3(a.batch), dim3(reg_tpb(n)), 0, s, a); break;
    SRBD_REGN_HORIZONS(SRBD_CASE)
#undef SRBD_CASE
    default: break;
  }
}

void launch_step(int N, const FusedArgs& a, hipStream_t s) {
  switch (N) {
#define SRBD_CASE(n) \
  case n: hipLaunchKernelGGL(mpc_step_reg_kernel<n>, dim3(a.batch), dim3(reg_tpb(n)), 0, s, a); break;
    SRBD_REGN_HORIZONS(SRBD_CASE)
#undef SRBD_CASE
    default: break;
  }
}

static_assert(reg_horizon(2) && reg_horizon(32) && !reg_horizon(33) && !reg_horizon(1),
              "SRBD_REGN_HORIZONS lists exactly the register horizons other than 10 and 20");

}  // namespace regn
}  // namespace srbd
