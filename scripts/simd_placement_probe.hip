// simd_placement_probe.hip -- diagnostic: which SIMD each wave of a two-wave workgroup lands on, with the
// N = 20 register kernels' resources (128 threads, 36.6 KB static LDS, 4 workgroups per CU), and which
// workgroups share a CU at the same time. Each wave records HW_ID (wave / SIMD / CU / SE), XCC_ID and
// s_memrealtime at its start and end; the host prints, per CU, how the waves of resident workgroups
// pair up on SIMDs.   hipcc --offload-arch=gfx950 -O3 -o /tmp/simd_probe scripts/simd_placement_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

constexpr int kLdsDoubles = 36576 / 8;

__global__ __launch_bounds__(128, 2) void probe(unsigned* rec, int spin) {
  __shared__ double lds[kLdsDoubles];
  const int w = threadIdx.x >> 6;
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID, 32 bits
  const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // HW_REG_XCC_ID
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  double acc = threadIdx.x;
  for (int i = 0; i < spin; ++i) {  // keep the workgroup resident for a while (LDS + VALU)
    lds[(threadIdx.x + i) % kLdsDoubles] = acc;
    __syncthreads();
    acc = acc * 1.0000001 + lds[(threadIdx.x * 7 + i) % kLdsDoubles];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    unsigned* r = rec + 8 * (2 * blockIdx.x + w);
    r[0] = hw;
    r[1] = xcc;
    r[2] = (unsigned)t0;
    r[3] = (unsigned)(t0 >> 32);
    r[4] = (unsigned)t1;
    r[5] = (unsigned)(t1 >> 32);
    r[6] = acc > 1e300 ? 1u : 0u;
  }
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 4096, spin = argc > 2 ? atoi(argv[2]) : 2000;
  unsigned* d;
  hipMalloc(&d, sizeof(unsigned) * 8 * 2 * B);
  hipLaunchKernelGGL(probe, dim3(B), dim3(128), 0, 0, d, spin);
  hipLaunchKernelGGL(probe, dim3(B), dim3(128), 0, 0, d, spin);
  hipDeviceSynchronize();
  std::vector<unsigned> h(8 * 2 * B);
  hipMemcpy(h.data(), d, sizeof(unsigned) * h.size(), hipMemcpyDeviceToHost);
  // per workgroup: simd of wave 0 and wave 1, CU key, start time
  std::map<int, int> pair_hist;  // (simd0 * 4 + simd1) -> count
  std::map<unsigned long long, std::vector<int>> by_cu;
  for (int b = 0; b < B; ++b) {
    const unsigned h0 = h[16 * b], h1 = h[16 * b + 8];
    const int s0 = (h0 >> 4) & 3, s1 = (h1 >> 4) & 3;
    pair_hist[s0 * 4 + s1]++;
    // CU identity: XCC, SE (bits 13-15), SH (12), CU (8-11) of HW_ID
    const unsigned long long key = ((unsigned long long)(h[16 * b + 1] & 15) << 16) | ((h0 >> 8) & 0xFF);
    by_cu[key].push_back(b);
  }
  printf("workgroups %d; (simd of wave 0, simd of wave 1): count\n", B);
  for (auto& kv : pair_hist) printf("  (%d, %d): %d\n", kv.first / 4, kv.first % 4, kv.second);
  // per CU, the first 4 workgroups in start order: their wave-0 SIMDs
  std::map<int, int> chain_simd_load;  // how many of the first 4 resident workgroups put wave 0 on each SIMD
  int shown = 0;
  for (auto& kv : by_cu) {
    auto v = kv.second;
    std::sort(v.begin(), v.end(), [&](int a, int c) {
      unsigned long long ta = h[16 * a + 2] | ((unsigned long long)h[16 * a + 3] << 32);
      unsigned long long tc = h[16 * c + 2] | ((unsigned long long)h[16 * c + 3] << 32);
      return ta < tc;
    });
    int cnt[4] = {0, 0, 0, 0};
    for (int k = 0; k < 4 && k < (int)v.size(); ++k) cnt[(h[16 * v[k]] >> 4) & 3]++;
    int mx = 0;
    for (int s = 0; s < 4; ++s) mx = cnt[s] > mx ? cnt[s] : mx;
    chain_simd_load[mx]++;
    if (shown++ < 6) {
      printf("CU key %llx: %zu workgroups; first 4 (wave0 simd, wave1 simd, start):", kv.first, v.size());
      for (int k = 0; k < 4 && k < (int)v.size(); ++k)
        printf(" (%u,%u,%u)", (h[16 * v[k]] >> 4) & 3, (h[16 * v[k] + 8] >> 4) & 3, h[16 * v[k] + 2] & 0xFFFFF);
      printf("\n");
    }
  }
  printf("CUs by the largest number of first-round wave-0s on one SIMD: ");
  for (auto& kv : chain_simd_load) printf("%d -> %d CUs; ", kv.first, kv.second);
  printf("\n");
  // the same if each workgroup put its chain on the wave of the lower / the even SIMD id, or by the
  // parity rule s0 ^ s1
  for (int rule = 0; rule < 3; ++rule) {
    std::map<int, int> load;
    for (auto& kv : by_cu) {
      auto v = kv.second;
      std::sort(v.begin(), v.end(), [&](int a, int c) {
        unsigned long long ta = h[16 * a + 2] | ((unsigned long long)h[16 * a + 3] << 32);
        unsigned long long tc = h[16 * c + 2] | ((unsigned long long)h[16 * c + 3] << 32);
        return ta < tc;
      });
      int cnt[4] = {0, 0, 0, 0};
      for (int k = 0; k < 4 && k < (int)v.size(); ++k) {
        const int s0 = (h[16 * v[k]] >> 4) & 3, s1 = (h[16 * v[k] + 8] >> 4) & 3;
        int c = s0;
        if (rule == 0) c = s0 < s1 ? s0 : s1;
        if (rule == 1) c = (s1 & 1) == 0 && (s0 & 1) ? s1 : s0;
        if (rule == 2) c = ((s0 + s1) & 2) ? s1 : s0;
        cnt[c]++;
      }
      int mx = 0;
      for (int s = 0; s < 4; ++s) mx = cnt[s] > mx ? cnt[s] : mx;
      load[mx]++;
    }
    printf("rule %d: ", rule);
    for (auto& kv : load) printf("%d -> %d CUs; ", kv.first, kv.second);
    printf("\n");
  }
  return 0;
}
