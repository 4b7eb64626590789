/* dropin_evaluate.c -- thin CusADi-ABI library: exports exactly `evaluate`, the symbol a CusADi
 * function library exports (reference biped_pympc/cusadi/src/generateCUDACode.py:157-183) and that
 * CusadiFunction binds (CusadiFunction.py:34-35,43-46). Compiled once per CasADi Function name:
 *   -DSRBD_FN_FORMER -DSRBD_N=10                 -> libqp_former.so
 *   -DSRBD_FN_PDIPM  -DSRBD_N=10 -DSRBD_ITERS=5  -> libsparse_pdipm_multiple_iterations.so
 * and forwards to libsrbd_mpc.so (same directory, rpath $ORIGIN). */
#include "../../include/srbd_mpc.h"

#ifndef SRBD_N
#define SRBD_N 10
#endif
#ifndef SRBD_SHIM_ID
#define SRBD_SHIM_ID "0000000000000000"
#endif

/* build provenance: hash of this shim, its configuration and libsrbd_mpc.so's build id
 * (biped_pympc_amd/build.py _shim_hash), read from the file by build.py */
__attribute__((used)) static const char srbd_shim_id_tag[] = "srbd-shim-id:" SRBD_SHIM_ID;

float evaluate(const double* inputs[], double* work, double* outputs[], const int batch_size) {
#if defined(SRBD_FN_FORMER)
  return srbd_evaluate_qp_former(SRBD_N, inputs, work, outputs, batch_size);
#elif defined(SRBD_FN_PDIPM)
  return srbd_evaluate_pdipm(SRBD_N, SRBD_ITERS, inputs, work, outputs, batch_size);
#else
#error "define SRBD_FN_FORMER or SRBD_FN_PDIPM"
#endif
}
