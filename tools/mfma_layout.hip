// Lane layouts of the fp64 MFMAs (development probe): v_mfma_f64_16x16x4f64 and v_mfma_f64_4x4x4f64.
// Each lane's A and B operands are one-hot coded (A = 1 on exactly one lane and 0 elsewhere, B the
// same) so that the single nonzero output element shows which (A lane, B lane) pair feeds which
// output lane / register.  Prints, per MFMA shape, lines "a_lane b_lane -> out_lane[reg]" for every
// pair whose product lands somewhere.
//   hipcc --offload-arch=gfx950 -O2 tools/mfma_layout.hip -o tools/bin/mfma_layout
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void probe16(const int* pairs, int np, double* out) {
  const int lane = threadIdx.x;
  for (int q = 0; q < np; ++q) {
    const double a = lane == pairs[2 * q] ? 1.0 : 0.0;
    const double b = lane == pairs[2 * q + 1] ? 1.0 : 0.0;
    d4 c = {0.0, 0.0, 0.0, 0.0};
    c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[((size_t)q * 64 + lane) * 4 + r] = c[r];
  }
}

__global__ void probe4(const int* pairs, int np, double* out) {
  const int lane = threadIdx.x;
  for (int q = 0; q < np; ++q) {
    const double a = lane == pairs[2 * q] ? 1.0 : 0.0;
    const double b = lane == pairs[2 * q + 1] ? 1.0 : 0.0;
    double c = 0.0;
    c = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
    out[(size_t)q * 64 + lane] = c;
  }
}

int main() {
  std::vector<int> pairs;
  for (int a = 0; a < 64; ++a)
    for (int b = 0; b < 64; ++b) pairs.push_back(a), pairs.push_back(b);
  const int np = 64 * 64;
  int* dp;
  double* dout;
  hipMalloc(&dp, sizeof(int) * pairs.size());
  hipMalloc(&dout, sizeof(double) * np * 64 * 4);
  hipMemcpy(dp, pairs.data(), sizeof(int) * pairs.size(), hipMemcpyHostToDevice);
  std::vector<double> h((size_t)np * 64 * 4);
  hipLaunchKernelGGL(probe16, dim3(1), dim3(64), 0, 0, dp, np, dout);
  hipMemcpy(h.data(), dout, sizeof(double) * h.size(), hipMemcpyDeviceToHost);
  std::printf("# 16x16x4f64: a_lane b_lane -> out_lane reg\n");
  for (int q = 0; q < np; ++q)
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r)
        if (h[((size_t)q * 64 + l) * 4 + r] != 0.0)
          std::printf("16 %d %d -> %d %d\n", pairs[2 * q], pairs[2 * q + 1], l, r);
  hipLaunchKernelGGL(probe4, dim3(1), dim3(64), 0, 0, dp, np, dout);
  hipMemcpy(h.data(), dout, sizeof(double) * np * 64, hipMemcpyDeviceToHost);
  std::printf("# 4x4x4f64: a_lane b_lane -> out_lane\n");
  for (int q = 0; q < np; ++q)
    for (int l = 0; l < 64; ++l)
      if (h[(size_t)q * 64 + l] != 0.0) std::printf("4 %d %d -> %d\n", pairs[2 * q], pairs[2 * q + 1], l);
  hipFree(dp);
  hipFree(dout);
  return 0;
}
