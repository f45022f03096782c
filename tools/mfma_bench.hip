// mfma_bench.hip -- measures the sustained fp64 matrix (v_mfma_f64_16x16x4_f64) and
// vector (v_fma_f64) rates on this device, plus the clock held under the MFMA loop.
// Development tool: hipcc --offload-arch=gfx950 -O3 tools/mfma_bench.hip -o build/mfma_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void __launch_bounds__(256) mfma_loop(double* out, int iters, double seed) {
  d4 acc[NACC];
  for (int k = 0; k < NACC; ++k) acc[k] = d4{seed, 0, 0, 0};
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0;
  for (int k = 0; k < NACC; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    out[gridDim.x * blockDim.x + 2 * blockIdx.x] = (double)(t1 - t0);
    out[gridDim.x * blockDim.x + 2 * blockIdx.x + 1] = (double)(r1 - r0);
  }
}

template <int NACC>
__global__ void __launch_bounds__(256) fma_loop(double* out, int iters, double seed) {
  double acc[NACC];
  for (int k = 0; k < NACC; ++k) acc[k] = seed + k;
  const double a = 1.0000001, b = seed * 1e-9 + threadIdx.x * 1e-12;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) acc[k] = __builtin_fma(acc[k], a, b);
  }
  double s = 0;
  for (int k = 0; k < NACC; ++k) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  double* out;
  hipMalloc(&out, sizeof(double) * 1 << 24);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, auto kern, int blocks_per_cu, int iters, double flops_per_thread_iter) {
    const int grid = ncu * blocks_per_cu;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, 10, 1.0);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, iters, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)grid * 256 * iters * flops_per_thread_iter;
    std::vector<double> h(2 * grid);
    hipMemcpy(h.data(), out + (size_t)grid * 256, sizeof(double) * 2 * grid, hipMemcpyDeviceToHost);
    double clk = 0;
    int cnt = 0;
    for (int b = 0; b < grid; ++b)
      if (h[2 * b + 1] > 0) { clk += h[2 * b] / h[2 * b + 1] * 100.0; ++cnt; }
    printf("%-28s blocks/CU %d  %.3f ms  %.2f TFLOP/s  clock %.0f MHz\n", name, blocks_per_cu, ms, flops / ms / 1e9,
           cnt ? clk / cnt : 0.0);
  };
  // each MFMA: 2*16*16*4 = 2048 flop per wave = 32 flop per lane
  for (int bpc : {1, 2, 4}) {
    run("mfma_f64 NACC=4", mfma_loop<4>, bpc, 20000, 4 * 32.0);
    run("mfma_f64 NACC=8", mfma_loop<8>, bpc, 10000, 8 * 32.0);
    run("mfma_f64 NACC=16", mfma_loop<16>, bpc, 5000, 16 * 32.0);
  }
  for (int bpc : {1, 2, 4}) run("v_fma_f64 NACC=8", fma_loop<8>, bpc, 20000, 8 * 2.0);
  return 0;
}
