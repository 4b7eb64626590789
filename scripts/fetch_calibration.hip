// fetch_calibration.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths
// the SRBD kernels use (the guide calibrates only 16 B/lane streaming reads: FETCH_SIZE = 1/2 bytes).
// Each kernel moves a known byte count from / to a 1 GiB buffer (past the 256 MiB Infinity Cache):
//   read8  : coalesced 8 B/lane loads (global_load_dwordx2), the width of the solver's FP64 loads
//   read16 : coalesced 16 B/lane loads (the guide's calibrated case)
//   rowread8: 64 lanes reading one short row (452 doubles, the fused kernel's former-input rows) per wave
//   write8 : coalesced 8 B/lane stores (the solution rows)
// Build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib scripts/fetch_calibration.hip
// Run:   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib ; rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void read8(const double* __restrict__ a, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 12345.678) out[0] = s;  // keep the loads
}
__global__ void read16(const double2* __restrict__ a, size_t n2, double* out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}
// one wave per row of `w` doubles, rows contiguous (the batched (B, nnz) layout)
__global__ void rowread8(const double* __restrict__ a, int w, int rows, double* out) {
  const int row = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64, lane = threadIdx.x & 63;
  if (row >= rows) return;
  double s = 0.0;
  for (int e = lane; e < w; e += 64) s += a[(size_t)row * w + e];
  if (s == 12345.678) out[0] = s;
}
__global__ void write8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = 1.0;
}

int main() {
  const size_t bytes = (size_t)1 << 30, n = bytes / 8;
  double *a, *out;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(a, 0, bytes) != hipSuccess) return 1;
  const int rows = (int)(bytes / (452 * 8));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(read8, dim3(4096), dim3(256), 0, 0, a, n, out);
    hipLaunchKernelGGL(read16, dim3(4096), dim3(256), 0, 0, (const double2*)a, n / 2, out);
    hipLaunchKernelGGL(rowread8, dim3((rows + 3) / 4), dim3(256), 0, 0, a, 452, rows, out);
    hipLaunchKernelGGL(write8, dim3(4096), dim3(256), 0, 0, a, n);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("bytes per kernel: read8 %zu read16 %zu rowread8 %zu write8 %zu\n", bytes, bytes,
              (size_t)rows * 452 * 8, bytes);
  return 0;
}
