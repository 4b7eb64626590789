// srbd_mpc.hip -- libsrbd_mpc.so: HIP kernels (gfx950) + the C-ABI of include/srbd_mpc.h.
//
// The main translation unit; the N = 20 register kernels are built apart in srbd_reg20.hip when
// SRBD_SPLIT_REG20 is defined (the product build, biped_pympc_amd/build.py). The constant-memory
// tables (srbd_common.hpp) are compile-time initialised, so each unit's copy is identical.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/srbd_mpc.h"
#include "pdipm.hpp"
#include "pdipm_srbd.hpp"
#include "pdipm_srbd_reg.hpp"
#include "mpc_step_lds.hpp"
#include "qp_former.hpp"
#include "mpc_io.hpp"
#include "reg20.hpp"
#include "regN.hpp"
#include "device_state.hpp"

#ifndef SRBD_BUILD_ID
#define SRBD_BUILD_ID "0000000000000000"  // diagnostic builds outside biped_pympc_amd/build.py
#endif

namespace {

// "srbd-build-id:" + the 16-hex source hash (build.py source_hash); build.py reads it from the file
__attribute__((used)) const char kBuildIdTag[] = "srbd-build-id:" SRBD_BUILD_ID;

thread_local std::string g_last_error;

int set_error(int code, const char* what) {
  char buf[512];
  std::snprintf(buf, sizeof(buf), "%s (code %d: %s)", what, code,
                code > 0 ? hipGetErrorString((hipError_t)code) : "invalid argument");
  g_last_error = buf;
  return code;
}

constexpr int kFormerWaves = 4;
constexpr int kErrInvalid = (int)hipErrorInvalidValue;
// general solves of non-stage-invariant QPs in flight per device: one slot per workgroup the device
// can hold resident of any stage-invariant kernel (at most 8 QPs per CU: the N <= 10 register kernels)
constexpr int kMaxQpsPerCu = 8;

bool horizon_ok(int N) { return N >= 1 && N <= srbd::kMaxN; }

size_t solver_lds_bytes(int N) { return sizeof(double) * (size_t)srbd::SolverLayout(N).total; }
size_t fast_lds_bytes(int N) { return sizeof(double) * (size_t)srbd::FastLayout(N).total; }
constexpr size_t kRegLds10 = sizeof(double) * (size_t)srbd::RegLayout<10>::total;
constexpr size_t kRegLds20 = sizeof(double) * (size_t)srbd::RegLayout<20>::total;
// the register kernels' LDS is static (RegLayout<N>::total doubles per workgroup)
static_assert(kRegLds10 <= 20 * 1024, "N=10 register kernel must fit 8 QPs per CU");
static_assert(kRegLds20 <= 40 * 1024, "N=20 register kernel must fit 4 QPs per CU");

// The HIP device current at this call (-1 if none / out of range for the per-device state)
int current_device() {
  int d = -1;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= srbd::kMaxDevices) return -1;
  return d;
}

// Solver path per device: 0 = auto (stage-invariant kernels -- register-resident for N = 10 and 20,
// LDS-resident otherwise -- and the general kernel for flagged QPs); 1 = general kernel only;
// 2 = LDS-resident fast kernel. Selected by srbd_set_solver_path for the current device.
srbd::PerDevice<int> g_solver_path;
int solver_path() {
  const int* p = g_solver_path.at(current_device());
  return p ? *p : 0;
}

// Refinement policy per device (srbd_set_refinement / srbd_set_refinement_policy). Mode 0 (default):
// the affine direction at a solve's initial iterate and on ill-conditioned iterates (the policy word
// below), the combined one in every iteration; mode 1: both in every iteration; mode 2: a policy word set
// by srbd_set_refinement_policy. Read by the register kernels only (the LDS-resident and general kernels
// refine both directions in every iteration).
struct RefinePolicy {
  int mode = 0;
  int flags = 0;
  double w = 0.0;
};
// mode 0's policy: the predictor at a solve's initial iterate (all z = 1) and in every iteration with
// z / s >= 1e4 in some row (round 6, DESIGN.md 3.3: with correctly rounded reciprocals, about round 5's
// N = 10 time for 23 -> 4 failing _ccs-campaign cases of 6657)
constexpr int kDefaultRefineFlags = SRBD_REFINE_AFFINE_AT_INIT;
constexpr double kDefaultRefineW = 1e4;
srbd::PerDevice<RefinePolicy> g_refinement;
int refinement_mode() {
  const RefinePolicy* p = g_refinement.at(current_device());
  return p ? p->mode : 0;
}
// the kernel arguments of the policy in effect: the word and the W threshold
template <class Args>
void set_refinement_args(Args& a) {
  const RefinePolicy* p = g_refinement.at(current_device());
  const int mode = p ? p->mode : 0;
  a.refine_policy = mode == 2 ? p->flags : (mode == 1 ? SRBD_REFINE_AFFINE_ALL : kDefaultRefineFlags);
  const double w = mode == 2 ? p->w : kDefaultRefineW;
  a.refine_w = w > 0.0 ? w : INFINITY;
}

int ensure_lds_attr(const void* fn, size_t bytes, srbd::LdsAttr& cache) {
  const int dev = current_device();
  if (dev < 0) return set_error((int)hipErrorInvalidDevice, "no current HIP device (or index >= 64)");
  if (!cache.claim(dev, bytes)) return 0;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) return set_error((int)e, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  cache.commit(dev, bytes);
  return 0;
}

int launch_former(const srbd::FormerArgs& a, hipStream_t s) {
  if (a.batch == 0) return 0;
  const int grid = (a.batch + kFormerWaves - 1) / kFormerWaves;
  hipLaunchKernelGGL(srbd::qp_former_kernel<kFormerWaves>, dim3(grid), dim3(64 * kFormerWaves), 0, s, a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error((int)e, "qp_former_kernel launch");
}

// The per-device scratch pool of the stage-invariant solver kernels (pdipm.hpp
// pdipm_general_scratch): CUs x kMaxQpsPerCu slots of general_slot_doubles() (2048 slots of
// srbd_scratch_slot_bytes() = 162,000 B: 332 MB of the 288 GB on an MI355X) and their lock words, one
// per 128-byte line, allocated on the first stage-invariant solver call on a device (or
// srbd_prepare_device) and kept until srbd_release_device. With a slot for every resident workgroup
// no fallback solve waits for another: a batch of QPs that are all not stage-invariant runs at the
// general solve's rate instead of queueing on a few slots. srbd_set_scratch_slots (or the
// SRBD_SCRATCH_SLOTS environment variable, read when the pool is allocated) caps the slot count, for
// processes that share a GPU: a fallback QP that finds every slot taken waits for one (the holders are
// resident workgroups, so they finish), which is correct at any count >= 1, only slower.
struct ScratchPool {
  double* buf = nullptr;
  int* locks = nullptr;
  int slots = 0;
  int stride = 0;  // doubles per slot
};

// doubles one slot needs: the general solve's layout at its largest horizon (not necessarily N = kMaxN:
// the precomputed couplings are dropped where they would not fit 160 KiB of LDS)
int general_slot_doubles() {
  int s = 0;
  for (int n = 1; n <= srbd::kMaxN; ++n) {  // (KX, the last array, is the general kernel's only)
    const srbd::SolverLayout L(n);
    s = std::max(s, L.KX >= 0 ? L.KX : L.total);
  }
  return s;
}
srbd::PerDevice<ScratchPool> g_scratch;
srbd::PerDevice<int> g_scratch_cap;  // srbd_set_scratch_slots per device; 0 = default
std::mutex g_scratch_mu;
// A solver launch holds g_pool_rw shared from attaching the pool to its arguments until the kernel is
// enqueued; srbd_release_device / a resizing srbd_set_scratch_slots take it exclusively before their
// hipDeviceSynchronize, so a pool is never freed between another thread's attach and its launch (the
// kernel would run on freed HBM). Lock order: g_pool_rw, then g_scratch_mu.
std::shared_mutex g_pool_rw;

// slots of a new pool on device `dev` with `cus` compute units
int pool_slots(int dev, int cus) {
  const int* capp = g_scratch_cap.at(dev);
  int cap = capp ? *capp : 0;
  if (cap <= 0)
    if (const char* env = std::getenv("SRBD_SCRATCH_SLOTS")) cap = std::atoi(env);
  return cap > 0 ? std::min(cap, 1 << 16) : cus * kMaxQpsPerCu;
}

// frees the pool of `pool` after the device has drained (g_scratch_mu held)
int release_pool(ScratchPool* pool) {
  if (!pool || !pool->buf) return 0;
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return set_error((int)e, "srbd_release_device: device synchronisation");
  (void)hipFree(pool->buf);
  (void)hipFree(pool->locks);
  *pool = ScratchPool{};
  return 0;
}

// the current device's pool, allocated on first use (`s`: the stream of the calling launch, checked for
// capture; null from srbd_prepare_device)
ScratchPool* scratch_pool(hipStream_t s, bool check_capture, int& rc) {
  rc = 0;
  const int dev = current_device();
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  ScratchPool* pool = g_scratch.at(dev);
  if (!pool) {
    rc = set_error((int)hipErrorInvalidDevice, "no current HIP device (or index >= 64)");
    return nullptr;
  }
  if (!pool->buf) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (check_capture && hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone) {
      rc = set_error(kErrInvalid, "srbd solver: first call on this device inside a stream capture (the "
                                  "scratch pool is allocated on first use: call srbd_prepare_device() first)");
      return nullptr;
    }
    const size_t per_slot = (size_t)general_slot_doubles();
    int cus = 0;
    hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int slots = pool_slots(dev, e == hipSuccess && cus > 0 ? cus : 256);
    const size_t lock_ints = (size_t)slots * srbd::kLockStride;
    double* buf = nullptr;
    int* locks = nullptr;
    if (e == hipSuccess) e = hipMalloc(&buf, sizeof(double) * per_slot * slots);
    if (e == hipSuccess) e = hipMalloc(&locks, sizeof(int) * lock_ints);
    if (e == hipSuccess) e = hipMemset(locks, 0, sizeof(int) * lock_ints);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
      (void)hipFree(buf);
      (void)hipFree(locks);
      rc = set_error((int)e, "srbd solver: scratch pool allocation");
      return nullptr;
    }
    pool->buf = buf;
    pool->locks = locks;
    pool->slots = slots;
    pool->stride = (int)per_slot;
  }
  return pool;
}

int attach_scratch(srbd::SolverArgs& a, hipStream_t s) {
  int rc = 0;
  ScratchPool* pool = scratch_pool(s, true, rc);
  if (!pool) return rc;
  a.scratch = pool->buf;
  a.scratch_locks = pool->locks;
  a.scratch_slots = pool->slots;
  a.scratch_stride = pool->stride;
  return 0;
}

int launch_solver(const srbd::SolverArgs& a0, hipStream_t s) {
  if (a0.batch == 0) return 0;
  static srbd::LdsAttr cfg_general, cfg_fast, cfg_fast10, cfg_fast20;
  srbd::SolverArgs a = a0;
  set_refinement_args(a);
  const int path = solver_path();
  std::shared_lock<std::shared_mutex> keep_pool(g_pool_rw);  // until the launch is enqueued
  // the stage-invariant kernels solve any other QP of the batch in the same launch (scratch pool)
  if (path != 1)
    if (int rc = attach_scratch(a, s)) return rc;
  if (path == 0 && srbd::regn::supported(a.N)) {  // the register kernel of another horizon
    srbd::regn::launch_solver(a.N, a, s);  // static LDS (RegLayout)
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_error((int)e, "pdipm_srbd_reg_kernel launch");
  }
  if (path == 0 && (a.N == 10 || a.N == 20)) {
    if (a.N == 10) {
      hipLaunchKernelGGL(srbd::pdipm_srbd_reg_kernel<10>, dim3(a.batch), dim3(64), 0, s, a);
    } else {
#ifdef SRBD_SPLIT_REG20
      srbd::reg20::launch_solver(a, s);
#else
      hipLaunchKernelGGL(srbd::pdipm_srbd_reg_kernel<20>, dim3(a.batch), dim3(srbd::reg_tpb(20)), 0, s, a);
#endif
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_error((int)e, "pdipm_srbd_reg_kernel launch");
  }
  if (path == 0 || path == 2) {
    const size_t lds = fast_lds_bytes(a.N);
    if (lds > 160 * 1024) return set_error(kErrInvalid, "horizon too large for the LDS-resident solver");
    // horizon-specialised instantiations for the common horizons, runtime-N otherwise
    const void* fn = a.N == 10 ? (const void*)srbd::pdipm_srbd_kernel<10>
                   : a.N == 20 ? (const void*)srbd::pdipm_srbd_kernel<20>
                               : (const void*)srbd::pdipm_srbd_kernel<0>;
    srbd::LdsAttr& cfg = a.N == 10 ? cfg_fast10 : a.N == 20 ? cfg_fast20 : cfg_fast;
    if (int rc = ensure_lds_attr(fn, lds, cfg)) return rc;
    if (a.N == 10) hipLaunchKernelGGL(srbd::pdipm_srbd_kernel<10>, dim3(a.batch), dim3(64), lds, s, a);
    else if (a.N == 20) hipLaunchKernelGGL(srbd::pdipm_srbd_kernel<20>, dim3(a.batch), dim3(64), lds, s, a);
    else hipLaunchKernelGGL(srbd::pdipm_srbd_kernel<0>, dim3(a.batch), dim3(64), lds, s, a);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : set_error((int)e, "pdipm_srbd_kernel launch");
  }
  const size_t lds = solver_lds_bytes(a.N);
  if (lds > 160 * 1024) return set_error(kErrInvalid, "horizon too large for the LDS-resident solver");
  if (int rc = ensure_lds_attr((const void*)srbd::pdipm_kernel, lds, cfg_general)) return rc;
  hipLaunchKernelGGL(srbd::pdipm_kernel, dim3(a.batch), dim3(srbd::kGeneralThreads), lds, s, a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error((int)e, "pdipm_kernel launch");
}

// CusADi-style blocking call on the legacy default stream, timed with hipEvents (one event pair
// per device, created on first use there; the reference creates and leaks two per call).
template <class F>
float timed_blocking(F&& launch) {
  struct Events {
    hipEvent_t ev[2];
  };
  static std::mutex mu;
  static srbd::PerDevice<Events> events;
  std::lock_guard<std::mutex> lock(mu);
  Events* ev = events.at(current_device());
  if (!ev) {
    set_error((int)hipErrorInvalidDevice, "no current HIP device (or index >= 64)");
    return -1.0f;
  }
  if (!ev->ev[0]) {
    if (hipEventCreate(&ev->ev[0]) != hipSuccess || hipEventCreate(&ev->ev[1]) != hipSuccess) {
      set_error((int)hipErrorInitializationError, "hipEventCreate");
      return -1.0f;
    }
  }
  (void)hipEventRecord(ev->ev[0], 0);
  if (launch() != 0) return -1.0f;
  (void)hipEventRecord(ev->ev[1], 0);
  hipError_t e = hipEventSynchronize(ev->ev[1]);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    set_error((int)e, "kernel execution");
    return -1.0f;
  }
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, ev->ev[0], ev->ev[1]);
  return ms / 1000.0f;
}

}  // namespace

extern "C" {

int srbd_abi_version(void) { return SRBD_ABI_VERSION; }

const char* srbd_build_id(void) { return kBuildIdTag + sizeof("srbd-build-id:") - 1; }

const char* srbd_last_error(void) { return g_last_error.c_str(); }

size_t srbd_solver_lds_bytes(int horizon) { return horizon_ok(horizon) ? solver_lds_bytes(horizon) : 0; }

int srbd_set_solver_path(int path) {
  if (path < 0 || path > 2)
    return set_error(kErrInvalid, "srbd_set_solver_path: 0 (auto), 1 (general) or 2 (LDS-resident fast)");
  int* p = g_solver_path.at(current_device());
  if (!p) return set_error((int)hipErrorInvalidDevice, "srbd_set_solver_path: no current HIP device");
  *p = path;
  return 0;
}

int srbd_get_solver_path(void) { return solver_path(); }

int srbd_set_refinement(int mode) {
  if (mode < 0 || mode > 1)
    return set_error(kErrInvalid, "srbd_set_refinement: 0 (ill-conditioned iterates) or 1 (every iteration)");
  RefinePolicy* p = g_refinement.at(current_device());
  if (!p) return set_error((int)hipErrorInvalidDevice, "srbd_set_refinement: no current HIP device");
  *p = RefinePolicy{mode, 0, 0.0};
  return 0;
}

int srbd_set_refinement_policy(int flags, double w) {
  const int known = SRBD_REFINE_AFFINE_ALL | SRBD_REFINE_AFFINE_AT_INIT | SRBD_REFINE_AFFINE_FIRST(255) |
                    SRBD_REFINE_AFFINE_LAST(255);
  if ((flags & ~known) != 0 || w != w)
    return set_error(kErrInvalid, "srbd_set_refinement_policy: unknown policy bits or a NaN threshold");
  RefinePolicy* p = g_refinement.at(current_device());
  if (!p) return set_error((int)hipErrorInvalidDevice, "srbd_set_refinement_policy: no current HIP device");
  *p = RefinePolicy{2, flags, w};
  return 0;
}

int srbd_get_refinement(void) { return refinement_mode(); }

int srbd_prepare_device(void) {
  int rc = 0;
  return scratch_pool(nullptr, false, rc) ? 0 : rc;
}

int srbd_release_device(void) {
  std::unique_lock<std::shared_mutex> no_launch(g_pool_rw);
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  ScratchPool* pool = g_scratch.at(current_device());
  if (!pool) return set_error((int)hipErrorInvalidDevice, "srbd_release_device: no current HIP device");
  return release_pool(pool);
}

int srbd_set_scratch_slots(int slots) {
  if (slots < 0) return set_error(kErrInvalid, "srbd_set_scratch_slots: slots >= 0 (0 = one per resident workgroup)");
  std::unique_lock<std::shared_mutex> no_launch(g_pool_rw);
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  const int dev = current_device();
  int* cap = g_scratch_cap.at(dev);
  ScratchPool* pool = g_scratch.at(dev);
  if (!cap || !pool) return set_error((int)hipErrorInvalidDevice, "srbd_set_scratch_slots: no current HIP device");
  *cap = slots;
  if (pool->buf) {  // re-sized on the next solver call (or srbd_prepare_device)
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (pool_slots(dev, cus) != pool->slots) return release_pool(pool);
  }
  return 0;
}

size_t srbd_scratch_pool_bytes(void) {
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  const ScratchPool* pool = g_scratch.at(current_device());
  if (!pool || !pool->buf) return 0;
  return sizeof(double) * (size_t)pool->stride * pool->slots + sizeof(int) * (size_t)pool->slots * srbd::kLockStride;
}

int srbd_scratch_pool_slots(void) {
  std::lock_guard<std::mutex> lock(g_scratch_mu);
  const ScratchPool* pool = g_scratch.at(current_device());
  return pool ? pool->slots : 0;
}

size_t srbd_scratch_slot_bytes(void) { return sizeof(double) * (size_t)general_slot_doubles(); }

size_t srbd_mpc_workspace_doubles(int horizon, int batch) {
  if (!horizon_ok(horizon) || batch < 0) return 0;
  const size_t N = (size_t)horizon;
  return (size_t)batch * (24 * N + 24 * N + (122 * N - 24) + 14 * N + 28 * N + 16 * N);
}

float srbd_evaluate_qp_former(int horizon, const double* inputs[], double* work, double* outputs[],
                              int batch) {
  (void)work;
  if (!horizon_ok(horizon) || batch < 0 || !inputs || !outputs) {
    set_error(kErrInvalid, "srbd_evaluate_qp_former: bad horizon/batch/pointer table");
    return -1.0f;
  }
  srbd::FormerArgs a{};
  a.dev_in = inputs;
  a.dev_out = outputs;
  a.N = horizon;
  a.batch = batch;
  return timed_blocking([&] { return launch_former(a, 0); });
}

float srbd_evaluate_pdipm(int horizon, int n_iter, const double* inputs[], double* work,
                          double* outputs[], int batch) {
  (void)work;
  if (!horizon_ok(horizon) || n_iter < 1 || batch < 0 || !inputs || !outputs) {
    set_error(kErrInvalid, "srbd_evaluate_pdipm: bad horizon/n_iter/batch/pointer table");
    return -1.0f;
  }
  srbd::SolverArgs a{};
  a.dev_in = inputs;
  a.dev_out = outputs;
  a.N = horizon;
  a.n_iter = n_iter;
  a.batch = batch;
  a.init_mode = 0;
  return timed_blocking([&] { return launch_solver(a, 0); });
}

int srbd_qp_former(int horizon, int batch, const double* const* inputs, double* const* outputs,
                   void* stream) {
  if (!horizon_ok(horizon) || batch < 0 || !inputs || !outputs)
    return set_error(kErrInvalid, "srbd_qp_former: bad arguments");
  if (batch == 0) return 0;  // empty batch: buffers may be null (zero-size allocations)
  srbd::FormerArgs a{};
  for (int i = 0; i < 17; ++i) {
    if (!inputs[i]) return set_error(kErrInvalid, "srbd_qp_former: null input");
    a.in[i] = inputs[i];
  }
  for (int i = 0; i < 6; ++i) {
    if (!outputs[i]) return set_error(kErrInvalid, "srbd_qp_former: null output");
    a.out[i] = outputs[i];
  }
  a.N = horizon;
  a.batch = batch;
  return launch_former(a, (hipStream_t)stream);
}

static int pdipm_common(int horizon, int n_iter, int batch, double y0, int init_mode,
                        const double* const* inputs, double* const* outputs, int* status, void* stream) {
  if (!horizon_ok(horizon) || n_iter < 1 || batch < 0 || !inputs || !outputs)
    return set_error(kErrInvalid, "srbd_pdipm: bad arguments");
  if (batch == 0) return 0;
  srbd::SolverArgs a{};
  const int nin = init_mode == 0 ? 10 : init_mode == 2 ? 7 : 6;  // QP + iterate / + x_init / QP only
  for (int i = 0; i < nin; ++i) {
    if (!inputs[i]) return set_error(kErrInvalid, "srbd_pdipm: null input");
    a.in[i] = inputs[i];
  }
  for (int i = 0; i < 6; ++i) {
    if (!outputs[i]) return set_error(kErrInvalid, "srbd_pdipm: null output");
    a.out[i] = outputs[i];
  }
  a.N = horizon;
  a.n_iter = n_iter;
  a.batch = batch;
  a.init_mode = init_mode;
  a.y0 = y0;
  a.status = status;
  return launch_solver(a, (hipStream_t)stream);
}

int srbd_pdipm(int horizon, int n_iter, int batch, const double* const* inputs,
               double* const* outputs, void* stream) {
  return pdipm_common(horizon, n_iter, batch, 0.0, 0, inputs, outputs, nullptr, stream);
}

int srbd_pdipm_cold(int horizon, int n_iter, int batch, double y0, const double* const* inputs,
                    double* const* outputs, void* stream) {
  return pdipm_common(horizon, n_iter, batch, y0, 1, inputs, outputs, nullptr, stream);
}

int srbd_pdipm_ccs(int horizon, int n_iter, int batch, const double* const* inputs, double* const* outputs,
                   void* stream) {
  if (!inputs || (batch > 0 && !inputs[6])) return set_error(kErrInvalid, "srbd_pdipm_ccs: null x_init");
  return pdipm_common(horizon, n_iter, batch, 0.0, 2, inputs, outputs, nullptr, stream);
}

int srbd_pdipm_ex(int horizon, int n_iter, int batch, int init_mode, double y0, const double* const* inputs,
                  double* const* outputs, int* status, void* stream) {
  if (init_mode < 0 || init_mode > 2) return set_error(kErrInvalid, "srbd_pdipm_ex: init_mode 0, 1 or 2");
  if (init_mode == 2 && (!inputs || (batch > 0 && !inputs[6])))
    return set_error(kErrInvalid, "srbd_pdipm_ex: null x_init");
  return pdipm_common(horizon, n_iter, batch, init_mode == 1 ? y0 : 0.0, init_mode, inputs, outputs, status, stream);
}

static int mpc_solve_two_kernels(int horizon, int n_iter, int batch, double y0, const double* const* former_inputs,
                                 double* qp_workspace, double* const* outputs, int* status, void* stream) {
  if (!horizon_ok(horizon) || !qp_workspace) return set_error(kErrInvalid, "srbd_mpc_solve: bad arguments");
  const size_t N = (size_t)horizon, B = (size_t)(batch < 0 ? 0 : batch);
  double* H = qp_workspace;
  double* f = H + B * 24 * N;
  double* A = f + B * 24 * N;
  double* b = A + B * (122 * N - 24);
  double* G = b + B * 14 * N;
  double* d = G + B * 28 * N;
  double* qp[6] = {H, f, A, b, G, d};
  if (int rc = srbd_qp_former(horizon, batch, former_inputs, qp, stream)) return rc;
  const double* sin[10] = {H, G, A, f, d, b, nullptr, nullptr, nullptr, nullptr};
  return pdipm_common(horizon, n_iter, batch, y0, 1, sin, outputs, status, stream);
}

int srbd_mpc_solve(int horizon, int n_iter, int batch, double y0, const double* const* former_inputs,
                   double* qp_workspace, double* const* outputs, void* stream) {
  return mpc_solve_two_kernels(horizon, n_iter, batch, y0, former_inputs, qp_workspace, outputs, nullptr, stream);
}

// launch of the fused / controller-step kernel (a fully set up FusedArgs): the register kernels at
// the horizons they are instantiated for (10, 20 and regN.hpp's), the LDS-resident one-launch step
// (mpc_step_lds.hpp) at every other horizon
static int launch_step(const srbd::FusedArgs& a0, hipStream_t st) {
  static srbd::LdsAttr cfg_lds;
  srbd::FusedArgs a = a0;
  set_refinement_args(a);
  if (srbd::regn::supported(a.N)) {
    srbd::regn::launch_step(a.N, a, st);  // static LDS (RegLayout)
  } else if (a.N != 10 && a.N != 20) {
    const size_t lds = srbd::step_lds_bytes(a.N);
    if (lds > 160 * 1024) return set_error(kErrInvalid, "horizon too large for the one-launch step");
    if (int rc = ensure_lds_attr((const void*)srbd::mpc_step_lds_kernel<0>, lds, cfg_lds)) return rc;
    hipLaunchKernelGGL(srbd::mpc_step_lds_kernel<0>, dim3(a.batch), dim3(64), lds, st, a);
  } else if (a.N == 10) {
    hipLaunchKernelGGL(srbd::mpc_step_reg_kernel<10>, dim3(a.batch), dim3(64), 0, st, a);
  } else {
#ifdef SRBD_SPLIT_REG20
    srbd::reg20::launch_step(a, st);
#else
    hipLaunchKernelGGL(srbd::mpc_step_reg_kernel<20>, dim3(a.batch), dim3(srbd::reg_tpb(20)), 0, st, a);
#endif
  }
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error((int)e, "mpc_step_reg_kernel launch");
}

int srbd_mpc_solve_fused_ex(int horizon, int n_iter, int batch, double y0, const double* const* former_inputs,
                            double* qp_workspace, double* const* outputs, int* status, void* stream) {
  if (!horizon_ok(horizon)) return set_error(kErrInvalid, "srbd_mpc_solve_fused: bad horizon");
  if (solver_path() != 0) {  // a non-auto solver path: former + that solver kernel
    if (!qp_workspace) return set_error(kErrInvalid, "srbd_mpc_solve_fused: a non-auto solver path needs qp_workspace");
    return mpc_solve_two_kernels(horizon, n_iter, batch, y0, former_inputs, qp_workspace, outputs, status, stream);
  }
  if (n_iter < 1 || batch < 0 || !former_inputs || !outputs)
    return set_error(kErrInvalid, "srbd_mpc_solve_fused: bad arguments");
  if (batch == 0) return 0;
  const size_t N = (size_t)horizon, B = (size_t)batch;
  srbd::FusedArgs a{};
  for (int i = 0; i < 17; ++i) {
    if (!former_inputs[i]) return set_error(kErrInvalid, "srbd_mpc_solve_fused: null input");
    a.in[i] = former_inputs[i];
  }
  for (int i = 0; i < 6; ++i) a.out[i] = outputs[i];  // null: not written
  if (qp_workspace) {  // same slots as srbd_mpc_solve's H, f, A, b, G, d
    a.vec[0] = qp_workspace + B * 24 * N;
    a.vec[1] = a.vec[0] + B * 24 * N + B * (122 * N - 24);
    a.vec[2] = a.vec[1] + B * 14 * N + B * 28 * N;
  }
  a.N = horizon;
  a.n_iter = n_iter;
  a.batch = batch;
  a.y0 = y0;
  a.status = status;
  return launch_step(a, (hipStream_t)stream);
}

int srbd_mpc_solve_fused(int horizon, int n_iter, int batch, double y0, const double* const* former_inputs,
                         double* qp_workspace, double* const* outputs, void* stream) {
  return srbd_mpc_solve_fused_ex(horizon, n_iter, batch, y0, former_inputs, qp_workspace, outputs, nullptr, stream);
}

// srbd_mpc_prep (host struct of device pointers + constants) -> the kernels' PrepArgs
static int fill_prep(const srbd_mpc_prep* p, srbd::PrepArgs& a, const char* who) {
  if (!p->root_euler || !p->root_position || !p->root_angular_velocity_w || !p->root_velocity_w ||
      !p->rotation_body || !p->foot_position || !p->desired_velocity_b || !p->desired_angular_velocity_b ||
      !p->desired_height || !p->world_position_desired || !p->yaw_desired || !p->first_run || !p->dt_mpc ||
      !p->residual_lin_accel || !p->residual_ang_accel ||
      (p->gait_phase ? (!p->ssp_durations || !p->dsp_durations) : !p->contact_table) ||
      (p->q_len != 12 && p->q_len != 13)) {
    std::string w = std::string(who) + ": missing array or bad q_len";
    return set_error(kErrInvalid, w.c_str());
  }
  a.root_euler = p->root_euler;
  a.root_position = p->root_position;
  a.ang_vel_w = p->root_angular_velocity_w;
  a.vel_w = p->root_velocity_w;
  a.rotation_body = p->rotation_body;
  a.foot_position = p->foot_position;
  a.des_vel_b = p->desired_velocity_b;
  a.des_angvel_b = p->desired_angular_velocity_b;
  a.des_height = p->desired_height;
  a.wpd = p->world_position_desired;
  a.yaw_des = p->yaw_desired;
  a.first_run = p->first_run;
  a.gait_phase = p->gait_phase;
  a.ssp = p->ssp_durations;
  a.dsp = p->dsp_durations;
  a.contact_table = p->contact_table;
  a.dt_mpc = p->dt_mpc;
  a.res_lin = p->residual_lin_accel;
  a.res_ang = p->residual_ang_accel;
  std::memcpy(a.I_body, p->I_body, sizeof(a.I_body));
  a.mass = p->mass;
  a.mu = p->mu;
  std::memcpy(a.Q, p->Q, sizeof(a.Q));
  a.q_len = p->q_len;
  std::memcpy(a.R, p->R, sizeof(a.R));
  a.step_dt = p->step_dt;
  a.literal = p->literal_layout ? 1 : 0;
  return 0;
}

int srbd_mpc_step_ex(int horizon, int n_iter, int batch, double y0, const srbd_mpc_prep* prep,
                     double* const* former_inputs, double* const* outputs, float* foot_wrench, int ndof,
                     const float* contact_jacobian, const float* contact_bool, float* tau, int* status,
                     void* stream) {
  if (!horizon_ok(horizon)) return set_error(kErrInvalid, "srbd_mpc_step: bad horizon");
  if (n_iter < 1 || batch < 0 || !prep || (tau && (ndof < 1 || ndof > 64)))
    return set_error(kErrInvalid, "srbd_mpc_step: bad arguments");
  if (batch == 0) return 0;
  if (!foot_wrench || (tau && (!contact_jacobian || !contact_bool)))
    return set_error(kErrInvalid, "srbd_mpc_step: null foot_wrench / contact_jacobian / contact_bool");
  srbd::FusedArgs a{};
  if (int rc = fill_prep(prep, a.prep, "srbd_mpc_step")) return rc;
  a.prep.N = horizon;
  a.prep.batch = batch;
  if (former_inputs)
    for (int i = 0; i < 17; ++i) {
      if (!former_inputs[i]) return set_error(kErrInvalid, "srbd_mpc_step: null former_inputs entry");
      a.prep.out[i] = former_inputs[i];
    }
  a.ctrl = 1;
  if (outputs)
    for (int i = 0; i < 6; ++i) a.out[i] = outputs[i];
  a.wrench = foot_wrench;
  a.tau = tau;
  a.jac = contact_jacobian;
  a.contact = contact_bool;
  a.ndof = tau ? ndof : 0;
  a.N = horizon;
  a.n_iter = n_iter;
  a.batch = batch;
  a.y0 = y0;
  a.status = status;
  return launch_step(a, (hipStream_t)stream);
}

int srbd_mpc_step(int horizon, int n_iter, int batch, double y0, const srbd_mpc_prep* prep,
                  double* const* former_inputs, double* const* outputs, float* foot_wrench, int ndof,
                  const float* contact_jacobian, const float* contact_bool, float* tau, void* stream) {
  return srbd_mpc_step_ex(horizon, n_iter, batch, y0, prep, former_inputs, outputs, foot_wrench, ndof,
                          contact_jacobian, contact_bool, tau, nullptr, stream);
}

int srbd_pattern_ccs(int horizon, int which, int* colptr, int* rowind) {
  if (!horizon_ok(horizon) || !colptr || !rowind) return -1;
  constexpr srbd::Tables T = srbd::make_tables();
  const int N = horizon, nz = 24 * N;
  int nnz = 0;
  std::vector<int> row, col;
  auto put = [&](int off, int r, int c) {
    if (off < 0 || off >= nnz) return false;
    if (row[off] != -1) return false;  // two entries mapped to one value slot
    row[off] = r;
    col[off] = c;
    return true;
  };
  if (which == 0) {
    nnz = nz;
    row.assign(nnz, -1);
    col.assign(nnz, -1);
    for (int c = 0; c < nz; ++c)
      if (!put(c, c, c)) return -2;
  } else if (which == 1) {
    nnz = srbd::nnz_A(N);
    row.assign(nnz, -1);
    col.assign(nnz, -1);
    for (int i = 0; i < N; ++i) {
      const int ub = srbd::a_ublock(N, i);
      for (int r = 0; r < 12; ++r) {
        if (!put(srbd::a_pidx(T, N, i, r), 12 * i + r, 12 * i + r)) return -2;  // x_{i+1}[r]
        for (int j = 0; j < 12; ++j) {
          if (i >= 1 && T.Mi[r][j] >= 0 && !put(srbd::a_xblock(i) + T.Mi[r][j], 12 * i + r, 12 * (i - 1) + j))
            return -2;
          if (T.Ni[r][j] >= 0 && !put(ub + T.Ni[r][j], 12 * i + r, 12 * N + 12 * i + j)) return -2;
        }
      }
      if (!put(ub + T.e6, 12 * N + 2 * i, 12 * N + 12 * i + 6)) return -2;
      if (!put(ub + T.e9, 12 * N + 2 * i + 1, 12 * N + 12 * i + 9)) return -2;
    }
  } else if (which == 2) {
    nnz = 28 * N;
    row.assign(nnz, -1);
    col.assign(nnz, -1);
    for (int i = 0; i < N; ++i)
      for (int q = 0; q < 28; ++q)
        if (!put(28 * i + q, 16 * i + T.grow[q], 12 * N + 12 * i + T.gcol[q])) return -2;
  } else {
    return -1;
  }
  // every slot filled, (col, row) strictly increasing in slot order  => valid sorted CCS
  for (int k = 0; k < nnz; ++k) {
    if (row[k] < 0) return -3;
    if (k > 0 && (col[k] < col[k - 1] || (col[k] == col[k - 1] && row[k] <= row[k - 1]))) return -4;
  }
  for (int c = 0; c <= nz; ++c) colptr[c] = 0;
  for (int k = 0; k < nnz; ++k) {
    colptr[col[k] + 1]++;
    rowind[k] = row[k];
  }
  for (int c = 0; c < nz; ++c) colptr[c + 1] += colptr[c];
  return nnz;
}

int srbd_prepare_inputs(int horizon, int batch, const srbd_mpc_prep* p, double* const* former_inputs,
                        void* stream) {
  if (!horizon_ok(horizon) || batch < 0 || !p || !former_inputs)
    return set_error(kErrInvalid, "srbd_prepare_inputs: bad arguments");
  if (batch == 0) return 0;
  srbd::PrepArgs a{};
  if (int rc = fill_prep(p, a, "srbd_prepare_inputs")) return rc;
  for (int i = 0; i < 17; ++i) {
    if (!former_inputs[i]) return set_error(kErrInvalid, "srbd_prepare_inputs: null output");
    a.out[i] = former_inputs[i];
  }
  a.N = horizon;
  a.batch = batch;
  hipLaunchKernelGGL(srbd::prepare_inputs_kernel, dim3((batch + 3) / 4), dim3(256), 0, (hipStream_t)stream, a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error((int)e, "prepare_inputs_kernel launch");
}

int srbd_u0_wrench(int horizon, int batch, const double* x, const float* rotation_body, float* foot_wrench,
                   void* stream) {
  return srbd_u0_wrench_torque(horizon, batch, x, rotation_body, foot_wrench, 0, nullptr, nullptr, nullptr, stream);
}

int srbd_u0_wrench_torque(int horizon, int batch, const double* x, const float* rotation_body, float* foot_wrench,
                          int ndof, const float* contact_jacobian, const float* contact_bool, float* tau,
                          void* stream) {
  const bool torque = tau != nullptr;
  if (!horizon_ok(horizon) || batch < 0 || (batch > 0 && (!x || !rotation_body || !foot_wrench)) ||
      (torque && (ndof < 1 || ndof > 64 || (batch > 0 && (!contact_jacobian || !contact_bool)))))
    return set_error(kErrInvalid, "srbd_u0_wrench_torque: bad arguments");
  if (batch == 0) return 0;
  hipLaunchKernelGGL(srbd::u0_wrench_kernel, dim3((batch + 255) / 256), dim3(256), 0, (hipStream_t)stream, horizon,
                     batch, x, rotation_body, foot_wrench, ndof, contact_jacobian, contact_bool, tau);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error((int)e, "u0_wrench_kernel launch");
}

int srbd_dense_scatter(int batch, int nnz, int rc, const int* inverse_index, const double* values, double* dense,
                       void* stream) {
  if (batch < 0 || nnz < 0 || rc < 0 || batch > 65535 ||
      (batch > 0 && rc > 0 && (!inverse_index || !dense || (nnz > 0 && !values))))
    return set_error(kErrInvalid, "srbd_dense_scatter: bad arguments (batch <= 65535 per call)");
  if (batch == 0 || rc == 0) return 0;
  hipLaunchKernelGGL(srbd::dense_scatter_kernel, dim3((rc + 511) / 512, batch), dim3(256), 0, (hipStream_t)stream, rc,
                     nnz, batch, (const int32_t*)inverse_index, values, dense);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_error((int)e, "dense_scatter_kernel launch");
}

}  // extern "C"
