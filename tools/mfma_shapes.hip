// mfma_shapes.hip -- sustained rate of the two fp64 MFMA shapes of gfx950 under the operand
// patterns the Gram kernels use: NACC independent accumulators, each MFMA with its own A / B
// registers (as the tile loops issue them), 1-4 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_shapes.hip -o tools/bin/mfma_shapes
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC, int NOP>
__global__ void __launch_bounds__(256) k16(double* out, int iters) {
  d4 acc[NACC];
  double a[NOP], b[NOP];
  for (int k = 0; k < NACC; ++k) acc[k] = d4{0.0, 0.0, 0.0, 0.0};
  for (int k = 0; k < NOP; ++k) {
    a[k] = 0.5 + 1e-3 * ((threadIdx.x * 7 + k * 13) & 63);
    b[k] = 0.5 - 1e-3 * ((threadIdx.x * 11 + k * 5) & 63);
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[k % NOP], b[(k + 1) % NOP], acc[k], 0, 0, 0);
  }
  double s = 0;
  for (int k = 0; k < NACC; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC, int NOP>
__global__ void __launch_bounds__(256) k4(double* out, int iters) {
  double acc[NACC], a[NOP], b[NOP];
  for (int k = 0; k < NACC; ++k) acc[k] = 0.0;
  for (int k = 0; k < NOP; ++k) {
    a[k] = 0.5 + 1e-3 * ((threadIdx.x * 7 + k * 13) & 63);
    b[k] = 0.5 - 1e-3 * ((threadIdx.x * 11 + k * 5) & 63);
  }
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < NACC; ++k) acc[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[k % NOP], b[(k + 1) % NOP], acc[k], 0, 0, 0);
  }
  double s = 0;
  for (int k = 0; k < NACC; ++k) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double* out;
  (void)hipMalloc(&out, 64 << 20);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto run = [&](const char* name, void (*kern)(double*, int), int blocks_per_cu, int iters, double flop_per_wave_iter) {
    const int grid = 256 * blocks_per_cu;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, 16);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)grid * 4 * iters * flop_per_wave_iter;
    printf("%-26s waves/SIMD %d  %8.3f ms  %6.1f TFLOP/s\n", name, blocks_per_cu, ms, flops / ms / 1e9);
  };
  for (int w : {1, 2, 4}) {
    run("16x16x4 NACC=4 NOP=4", k16<4, 4>, w, 20000, 4 * 2048.0);
    run("16x16x4 NACC=8 NOP=8", k16<8, 8>, w, 10000, 8 * 2048.0);
    run("16x16x4 NACC=10 NOP=5", k16<10, 5>, w, 8000, 10 * 2048.0);
    run("4x4x4   NACC=8 NOP=8", k4<8, 8>, w, 40000, 8 * 512.0);
    run("4x4x4   NACC=16 NOP=8", k4<16, 8>, w, 20000, 16 * 512.0);
  }
  return 0;
}
