// mfma_f64_layout.hip -- check the v_mfma_f64_16x16x4f64 operand / result lane maps on gfx950 with
// exact integer data (cdna_hip_programming.md: A[l&15][l>>4], B[l>>4][l&15], D[(l>>4)+4j][l&15]),
// and the accumulator-as-operand chain S = K + P (B P^T) the S_ii build uses.
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k(const double* A, const double* B, const double* Cm, double* D, double* S) {
  const int l = threadIdx.x;
  const double a = A[(l & 15) * 4 + (l >> 4)], b = B[(l >> 4) * 16 + (l & 15)];
  d4 c;
  for (int j = 0; j < 4; ++j) c[j] = Cm[((l >> 4) + 4 * j) * 16 + (l & 15)];
  d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int j = 0; j < 4; ++j) D[((l >> 4) + 4 * j) * 16 + (l & 15)] = d[j];
  // chain: P (16x8, rows >= 12 zero), Bm (8x8 in rows 0..7 of A-operand space), K (16x16)
  // U = Bm P^T (two k-steps), S = K + P U
  double pa[2], ba[2];
  for (int s = 0; s < 2; ++s) {
    const int r = l & 15, kk = 4 * s + (l >> 4);
    pa[s] = r < 12 ? (double)((r * 7 + kk * 3) % 5 - 2) : 0.0;      // P[r][kk]
    ba[s] = r < 8 ? (double)((r + 2 * kk) % 4 - 1) : 0.0;            // Bm[r][kk]
  }
  d4 u = {0, 0, 0, 0};
  for (int s = 0; s < 2; ++s) u = __builtin_amdgcn_mfma_f64_16x16x4f64(ba[s], pa[s], u, 0, 0, 0);
  d4 sacc;
  for (int j = 0; j < 4; ++j) sacc[j] = (double)(((l >> 4) + 4 * j) * 100 + (l & 15));
  for (int s = 0; s < 2; ++s) sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[s], u[s], sacc, 0, 0, 0);
  for (int j = 0; j < 4; ++j) S[((l >> 4) + 4 * j) * 16 + (l & 15)] = sacc[j];
}

int main() {
  double hA[64], hB[64], hC[256], hD[256], hS[256];
  for (int i = 0; i < 64; ++i) { hA[i] = (i * 3) % 7 - 3; hB[i] = (i * 5) % 9 - 4; }
  for (int i = 0; i < 256; ++i) hC[i] = i % 11;
  double *A, *B, *C, *D, *S;
  hipMalloc(&A, 512); hipMalloc(&B, 512); hipMalloc(&C, 2048); hipMalloc(&D, 2048); hipMalloc(&S, 2048);
  hipMemcpy(A, hA, 512, hipMemcpyHostToDevice); hipMemcpy(B, hB, 512, hipMemcpyHostToDevice);
  hipMemcpy(C, hC, 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, A, B, C, D, S);
  hipMemcpy(hD, D, 2048, hipMemcpyDeviceToHost); hipMemcpy(hS, S, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double r = hC[i * 16 + j];
      for (int q = 0; q < 4; ++q) r += hA[i * 4 + q] * hB[q * 16 + j];
      if (r != hD[i * 16 + j]) ++bad;
    }
  // host reference of the chain
  int bad2 = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double acc = i * 100 + j;
      for (int kk = 0; kk < 8; ++kk) {
        const double P_ik = i < 12 ? (double)((i * 7 + kk * 3) % 5 - 2) : 0.0;
        double U_kj = 0.0;  // U = Bm P^T: U[kk][j] = sum_m Bm[kk][m] P[j][m]
        for (int m = 0; m < 8; ++m) {
          const double Bm = (double)((kk + 2 * m) % 4 - 1);
          const double P_jm = j < 12 ? (double)((j * 7 + m * 3) % 5 - 2) : 0.0;
          U_kj += Bm * P_jm;
        }
        acc += P_ik * U_kj;
      }
      if (acc != hS[i * 16 + j]) ++bad2;
    }
  std::printf("mfma_f64_16x16x4 layout mismatches: %d / 256; chain S = K + P (B P^T) mismatches: %d / 256\n", bad, bad2);
  return bad || bad2;
}
