#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k16(double* out, int iters) {
  d4 acc[8];
  for (int k = 0; k < 8; ++k) acc[k] = d4{1.0 * k, 0, 0, 0};
  double a = 1.0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-3;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
  }
  double s = 0; for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
__global__ void __launch_bounds__(256) k4(double* out, int iters) {
  double acc[8];
  for (int k = 0; k < 8; ++k) acc[k] = 1.0 * k;
  double a = 1.0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-3;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[k], 0, 0, 0);
  }
  double s = 0; for (int k = 0; k < 8; ++k) s += acc[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
  double* out; hipMalloc(&out, 8 << 20);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000, grid = 1024;
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    hipEventRecord(e0); hipLaunchKernelGGL(k16, dim3(grid), dim3(256), 0, 0, out, iters); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double macs16 = (double)grid * 4 * iters * 8 * 1024;  // 4 waves/block, 1024 MACs per instr
    printf("16x16x4 f64: %.3f ms  %.1f TFLOP/s\n", ms, 2 * macs16 / ms / 1e9);
    hipEventRecord(e0); hipLaunchKernelGGL(k4, dim3(grid), dim3(256), 0, 0, out, iters); hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double macs4 = (double)grid * 4 * iters * 8 * 256;   // 4 blocks x 4x4x4 = 256 MACs per instr
    printf("4x4x4 f64 (4 blocks): %.3f ms  %.1f TFLOP/s\n", ms, 2 * macs4 / ms / 1e9);
  }
  return 0;
}
