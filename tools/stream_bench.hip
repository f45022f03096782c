// stream_bench.hip -- development tool: LDS-DMA streaming rate of the narrow pass's access
// pattern (column-major X, NRB-row column segments, 128/NRB columns per 1 KiB wave-instruction)
// against a row-block-major layout (each NRB x NC block contiguous), same bytes, per-wave
// pipelines DEPTH blocks deep, NW waves per workgroup, no compute.  Also reports the clock held
// (s_memtime vs s_memrealtime).
//   hipcc --offload-arch=gfx950 -O3 tools/stream_bench.hip -o build/stream_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void wait_vm_n(int n) {
  // n is a compile-time constant after unrolling at every call site below
  switch (n) {
#define W(N) case N: __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8)); break;
    W(0) W(4) W(8) W(12) W(16) W(24) W(32) W(48)
#undef W
    default: __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8)); break;
  }
}

template <int NRB, int NC, int DEPTH, int NW, bool BLOCKED, int AUX = 0>
__global__ void __launch_bounds__(64 * NW, 1) stream_kernel(const double* X, int64_t ld, int64_t nb, double* out,
                                                            unsigned long long* clk) {
  constexpr int NOCT = NC * NRB / 128;  // 1 KiB wave-instructions per block
  constexpr int CPI = 128 / NRB;        // columns per instruction
  __shared__ double lds[NW * DEPTH * NC * NRB];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double* wl = lds + wv * DEPTH * NC * NRB;
  const int64_t gw = (int64_t)blockIdx.x * NW + wv, nwt = (int64_t)gridDim.x * NW;
  const int64_t b0 = nb * gw / nwt, b1 = nb * (gw + 1) / nwt;
  const int cc = lane / (NRB / 2), j = lane % (NRB / 2);
  const int64_t loff = BLOCKED ? (int64_t)lane * 2 : (int64_t)cc * ld + 2 * j;
  auto stage = [&](int buf, int64_t blk) {
#pragma unroll
    for (int o = 0; o < NOCT; ++o) {
      const double* src =
          BLOCKED ? X + blk * (NC * NRB) + o * 128 + loff : X + blk * NRB + (int64_t)(CPI * o) * ld + loff;
      __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(wl + buf * NC * NRB + o * 128), 16, 0, AUX);
    }
  };
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double acc = 0.0;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (b0 + d < b1) stage(d, b0 + d);
  for (int64_t blk = b0; blk < b1; ++blk) {
    const int buf = (int)((blk - b0) % DEPTH);
    if (blk + DEPTH - 1 < b1) wait_vm_n(NOCT * (DEPTH - 1));
    else wait_vm_n(0);
    acc += wl[buf * NC * NRB + lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (blk + DEPTH < b1) stage(buf, blk + DEPTH);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 64 * NW + threadIdx.x] = acc;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

// Fill with random-looking doubles in (-1, 1): HBM / fabric power (and with it the sustained
// rate) depends on the data; an all-zero image measures an optimistic number.
__global__ void fill_kernel(double* x, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    x[i] = (double)(z >> 11) * 0x1.0p-52 - 1.0;
  }
}

static double* X;
static double* out;
static unsigned long long* clk;
static const int64_t NROWS = 400000000;  // 102 GB at 32 columns, 205 GB at 64

template <int NRB, int NC, int DEPTH, int NW, bool BLOCKED, int AUX = 0>
void run(int grid) {
  const int64_t n = NC == 32 ? NROWS : NROWS / 2, nb = n / NRB;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int it = 0; it < 4; ++it) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((stream_kernel<NRB, NC, DEPTH, NW, BLOCKED, AUX>), dim3(grid), dim3(64 * NW), 0, 0, X, n, nb, out, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[2];
    hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
    if (it == 3)
      printf("p %2d NRB %2d depth %d waves %2d grid %3d aux %d %s: %.3f ms  %.0f GB/s  clock %.2f GHz  LDS %d KiB\n", NC, NRB,
             DEPTH, NW, grid, AUX, BLOCKED ? "row-block-major" : "column-major   ", ms, (double)n * NC * 8 / ms / 1e6,
             (double)h[0] / (double)h[1] * 0.1, NW * DEPTH * NC * NRB * 8 / 1024);
  }
  fflush(stdout);
}

int main() {
  const size_t bytes = sizeof(double) * NROWS * 32;
  if (hipMalloc(&X, bytes) != hipSuccess) return 1;
  if (getenv("STREAM_ZERO")) hipMemset(X, 0, bytes);
  else hipLaunchKernelGGL(fill_kernel, dim3(65536), dim3(256), 0, 0, X, (int64_t)NROWS * 32);
  hipDeviceSynchronize();
  hipMalloc(&out, sizeof(double) * 512 * 1024);
  hipMalloc(&clk, sizeof(unsigned long long) * 2 * 512);
  // the cache policy of the DMA (aux: 0 default, 2 non-temporal as the IRLS passes use, 1 glc,
  // 3 glc + nt) on the narrow pass's two geometries
  run<32, 32, 2, 8, false, 0>(256);
  run<32, 32, 2, 8, false, 2>(256);
  run<32, 32, 2, 8, false, 1>(256);
  run<32, 32, 2, 8, false, 3>(256);
  run<16, 64, 2, 8, false, 0>(256);
  run<16, 64, 2, 8, false, 2>(256);
  run<16, 64, 2, 8, false, 1>(256);
  run<16, 64, 2, 8, false, 3>(256);
  // depth / waves at nt
  run<32, 32, 3, 4, false, 2>(256);
  run<16, 32, 4, 8, false, 2>(256);
  run<32, 32, 2, 4, false, 2>(512);
  return 0;
}
