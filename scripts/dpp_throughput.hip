// dpp_throughput.hip -- is v_fmac_f64_dpp's 8-cycle issue cost a per-wave latency or VALU-pipe
// occupancy? (diagnostic, gfx950). Each wave runs R rounds of 8 independent FMAs; the grid puts W
// waves on every SIMD (1024 W one-wave workgroups); if two waves per SIMD finish in the time of
// one, the cost is per-wave and the partner wave's instructions fill it.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/dpp_throughput scripts/dpp_throughput.hip
//   ./scripts/dpp_throughput
#include <hip/hip_runtime.h>
#include <stdio.h>

#define R8(OP) OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6") OP("%7")
#define DPP(X) "v_fmac_f64_dpp " X ", " X ", %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
#define PLAIN(X) "v_fmac_f64 " X ", " X ", %8\n"
#define MOVDPP(X) "v_mov_b64_dpp " X ", %8 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"

template <int MODE>
__global__ __launch_bounds__(64) void tput(double* out, int rounds, double c) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
         a7 = a0 + 7;
  for (int r = 0; r < rounds; ++r) {
    if constexpr (MODE == 0)
      asm volatile("s_nop 1\n" R8(DPP) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));
    else if constexpr (MODE == 1)
      asm volatile(R8(PLAIN) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));
    else
      asm volatile("s_nop 1\n" R8(MOVDPP) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c));
  }
  out[blockIdx.x * 64 + threadIdx.x] = ((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7));
}

int main() {
  const int rounds = 4096;
  double* out;
  hipMalloc(&out, sizeof(double) * 64 * 1024 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[3] = {"v_fmac_f64_dpp row_newbcast", "v_fmac_f64 (plain)", "v_mov_b64_dpp row_newbcast"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int W = 1; W <= 4; W *= 2) {
      const int grid = 1024 * W;
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        hipEventRecord(e0);
        if (mode == 0) tput<0><<<grid, 64>>>(out, rounds, 1e-9);
        else if (mode == 1) tput<1><<<grid, 64>>>(out, rounds, 1e-9);
        else tput<2><<<grid, 64>>>(out, rounds, 1e-9);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
      }
      // cycles per instruction per SIMD at the measured clock: instructions per SIMD = W * rounds * 8
      const double ns_per_inst = best * 1e6 / ((double)W * rounds * 8);
      printf("%-30s waves/SIMD %d: %.3f ms, %.3f ns per instruction per SIMD (%.1f cycles at 2.4 GHz)\n",
             names[mode], W, best, ns_per_inst, ns_per_inst * 2.4);
    }
  }
  hipFree(out);
  return 0;
}
