// stream_bench.hip -- development tool: LDS-DMA streaming rate of the narrow pass's access
// pattern (column-major X, NRB-row column segments, 8 columns per 1 KiB wave-instruction)
// against a row-block-major layout (each NRB x 64 block contiguous), same bytes, same
// double-buffered per-wave pipeline, no compute.  Also reports the clock held (s_memtime vs
// s_memrealtime).
//   hipcc --offload-arch=gfx950 -O3 tools/stream_bench.hip -o build/stream_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

constexpr int NRB = 16, NC = 64, NWAVE = 8, NOCT = NC * NRB / 128;

template <bool BLOCKED>
__global__ void __launch_bounds__(512, 1) stream_kernel(const double* X, int64_t ld, int64_t nb, double* out,
                                                        unsigned long long* clk) {
  __shared__ double lds[NWAVE * 2 * NC * NRB];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double* wl = lds + wv * 2 * NC * NRB;
  const int64_t gw = (int64_t)blockIdx.x * NWAVE + wv, nwt = (int64_t)gridDim.x * NWAVE;
  const int64_t b0 = nb * gw / nwt, b1 = nb * (gw + 1) / nwt;
  const int cc = lane >> 3, j = lane & 7;
  const int64_t loff = BLOCKED ? (int64_t)lane * 2 : (int64_t)cc * ld + 2 * j;
  auto stage = [&](int buf, int64_t blk) {
#pragma unroll
    for (int o = 0; o < NOCT; ++o) {
      const double* src = BLOCKED ? X + blk * (NC * NRB) + o * 128 + loff : X + blk * NRB + (int64_t)(8 * o) * ld + loff;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(wl + buf * NC * NRB + o * 128), 16, 0, 0);
    }
  };
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double acc = 0.0;
  if (b0 < b1) stage(0, b0);
  if (b0 + 1 < b1) stage(1, b0 + 1);
  for (int64_t blk = b0; blk < b1; ++blk) {
    const int buf = (int)((blk - b0) & 1);
    if (blk + 1 < b1) wait_vm<NOCT>();
    else wait_vm<0>();
    acc += wl[buf * NC * NRB + lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (blk + 2 < b1) stage(buf, blk + 2);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 512 + threadIdx.x] = acc;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  const int64_t n = 100000000;  // rows: 51.2 GB of fp64 X at 64 columns
  const int64_t nb = n / NRB;
  double* X;
  if (hipMalloc(&X, sizeof(double) * n * NC) != hipSuccess) return 1;
  hipMemset(X, 0, sizeof(double) * n * NC);
  double* out;
  unsigned long long* clk;
  hipMalloc(&out, sizeof(double) * 256 * 512);
  hipMalloc(&clk, sizeof(unsigned long long) * 512);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep)
    for (int blocked = 0; blocked < 2; ++blocked) {
      for (int it = 0; it < 4; ++it) {
        hipEventRecord(e0);
        if (blocked)
          hipLaunchKernelGGL(stream_kernel<true>, dim3(256), dim3(512), 0, 0, X, n, nb, out, clk);
        else
          hipLaunchKernelGGL(stream_kernel<false>, dim3(256), dim3(512), 0, 0, X, n, nb, out, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long h[2];
        hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
        if (it == 3)
          printf("%s: %.3f ms  %.0f GB/s  clock %.2f GHz\n", blocked ? "row-block-major" : "column-major   ", ms,
                 (double)n * NC * 8 / ms / 1e6, (double)h[0] / (double)h[1] * 0.1);
      }
    }
  return 0;
}
