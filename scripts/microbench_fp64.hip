// microbench_fp64.hip -- measured FP64 facts the solver kernels are designed around (gfx950).
// Build + run: python scripts/microbench_fp64.py  (GPU box). Results: profiles/r01/microbench_fp64.txt
//   acc_kernel:  max |x * r(x) - 1| of v_rcp_f64 alone, +1 and +2 Newton steps, and whether 1 NR
//                step reproduces the correctly rounded 1/x bit for bit
//   lat_kernel:  s_memtime cycles per link of a dependent chain (one wave): v_fma_f64,
//                v_mov_b64_dpp row_newbcast -> v_fma_f64, v_rcp_f64, ds_bpermute_b32 (x2, one double)
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" __global__ void acc_kernel(const double* x, int n, unsigned long long* out) {
  // out[0..2]: max |x r - 1| bits (as double bits, atomicMax on the bit pattern of a positive
  // double orders correctly); out[3]: count where 1-NR != 1/x; out[4]: count where 2-NR != 1/x
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double d = x[i];
  const double r0 = __builtin_amdgcn_rcp(d);
  const double r1 = fma(r0, fma(-d, r0, 1.0), r0);
  const double r2 = fma(r1, fma(-d, r1, 1.0), r1);
  const double ex = 1.0 / d;
  const double e0 = fabs(fma(d, r0, -1.0)), e1 = fabs(fma(d, r1, -1.0)), e2 = fabs(fma(d, r2, -1.0));
  atomicMax(&out[0], (unsigned long long)__double_as_longlong(e0));
  atomicMax(&out[1], (unsigned long long)__double_as_longlong(e1));
  atomicMax(&out[2], (unsigned long long)__double_as_longlong(e2));
  if (r1 != ex) atomicAdd(&out[3], 1ull);
  if (r2 != ex) atomicAdd(&out[4], 1ull);
  const double e = fma(-d, r0, 1.0), r3 = fma(r0, fma(e, e, e), r0);  // cubic step (rcp3)
  atomicMax(&out[5], (unsigned long long)__double_as_longlong(fabs(fma(d, r3, -1.0))));
  if (r3 != ex) atomicAdd(&out[6], 1ull);
}

#define CHAIN 256
extern "C" __global__ void lat_kernel(double seed, unsigned long long* cyc, double* sink) {
  double a = seed + threadIdx.x, b = 1.0000001, c = 1e-9;
  unsigned long long t0, t1;
  // 1. dependent v_fma_f64
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int k = 0; k < CHAIN; ++k) {
    a = fma(a, b, c);
    asm volatile("" : "+v"(a));
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
  // 2. DPP broadcast feeding an FMA
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int k = 0; k < CHAIN; ++k) {
    a = fma(__builtin_amdgcn_mov_dpp(a, 0x153, 0xF, 0xF, true), b, c);
    asm volatile("" : "+v"(a));
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[1] = t1 - t0;
  // 3. dependent v_rcp_f64
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int k = 0; k < CHAIN; ++k) {
    a = __builtin_amdgcn_rcp(a);
    asm volatile("" : "+v"(a));
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[2] = t1 - t0;
  // 4. ds_bpermute of a double (two b32) feeding an FMA
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 8
  for (int k = 0; k < CHAIN / 4; ++k) {
    a = fma(__shfl(a, (threadIdx.x + 16) & 63, 64), b, c);
    asm volatile("" : "+v"(a));
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[3] = (t1 - t0) * 4;
  // 5. independent v_fma_f64 throughput (8 chains)
  double v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int k = 0; k < CHAIN / 8; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = fma(v[j], b, c);
      asm volatile("" : "+v"(v[j]));
    }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[4] = t1 - t0;
  // 6. dependent DPP moves only
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int k = 0; k < CHAIN; ++k) {
    a = __builtin_amdgcn_mov_dpp(a, 0x153, 0xF, 0xF, true);
    asm volatile("" : "+v"(a));
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[5] = t1 - t0;
  // 7. independent v_mov_b64_dpp issue cost (8 independent sources)
  double w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = v[j];
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int k = 0; k < CHAIN / 8; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      w[j] = __builtin_amdgcn_mov_dpp(v[j], 0x150 + 3, 0xF, 0xF, true);
      asm volatile("" : "+v"(w[j]));
    }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[6] = t1 - t0;
  // 8. LDS broadcast round trip: lane 3 stores a double, everyone reads it back (dependent)
  __shared__ double buf[64];
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
  for (int k = 0; k < CHAIN / 8; ++k) {
    if (threadIdx.x == 3) buf[k & 7] = a;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    a = fma(buf[k & 7], b, c);
    asm volatile("" : "+v"(a));
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[7] = (t1 - t0) * 8;
  // 9. independent v_fmac_f64_dpp row_newbcast (8 accumulators, one asm block per round)
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int k = 0; k < CHAIN / 8; ++k) {
    asm volatile(
        "s_nop 1\n"
        "v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n"
        "v_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n"
        : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7])
        : "v"(a), "v"(b));
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[8] = t1 - t0;
  // 10. same 8 products as separate v_mov_b64_dpp + v_fmac_f64
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
  for (int k = 0; k < CHAIN / 8; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = fma(__builtin_amdgcn_mov_dpp(a, 0x151, 0xF, 0xF, true), b, v[j]);
      asm volatile("" : "+v"(v[j]));
    }
  }
  t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[9] = t1 - t0;
  double s = a;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += v[j] + w[j];
  sink[threadIdx.x] = s;
}

extern "C" int run_acc(const double* x, int n, unsigned long long* out) {
  hipLaunchKernelGGL(acc_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, x, n, out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
extern "C" int run_lat(unsigned long long* cyc, double* sink) {
  hipLaunchKernelGGL(lat_kernel, dim3(1), dim3(64), 0, 0, 1.0, cyc, sink);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
