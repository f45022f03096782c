// coexec_bench.hip -- do fp64 MFMA and fp64 VALU work overlap on one SIMD?  Waves 0-3 of a
// 512-thread workgroup run an MFMA loop, waves 4-7 (same SIMDs) an f64 FMA loop.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(512) mixed(double* out, int mfma_iters, int fma_iters, int int_iters) {
  const int wv = threadIdx.x >> 6;
  double s = 0;
  if (wv < 4) {
    d4 acc[8];
    for (int k = 0; k < 8; ++k) acc[k] = d4{1.0 * k, 0, 0, 0};
    double a = 1.0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-3;
    for (int i = 0; i < mfma_iters; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
    }
    for (int k = 0; k < 8; ++k) s += acc[k][0] + acc[k][3];
  } else {
    double acc[8];
    for (int k = 0; k < 8; ++k) acc[k] = 1.0 + k;
    const double a = 1.0000001, b = threadIdx.x * 1e-12;
    for (int i = 0; i < fma_iters; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = __builtin_fma(acc[k], a, b);
    }
    unsigned u = threadIdx.x;
    for (int i = 0; i < int_iters; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) u = u * 1664525u + 1013904223u;
    }
    for (int k = 0; k < 8; ++k) s += acc[k];
    s += u;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double* out;
  hipMalloc(&out, sizeof(double) << 22);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, int m, int f, int it) {
    hipLaunchKernelGGL(mixed, dim3(256), dim3(512), 0, 0, out, 10, 10, 10);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(mixed, dim3(256), dim3(512), 0, 0, out, m, f, it);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-34s %.3f ms\n", name, ms);
  };
  run("mfma only (4 waves)", 20000, 0, 0);
  run("f64 fma only (4 waves)", 0, 40000, 0);
  run("mfma + f64 fma", 20000, 40000, 0);
  run("int only (4 waves)", 0, 0, 40000);
  run("mfma + int", 20000, 0, 40000);
  return 0;
}
