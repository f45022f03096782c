// mfma44_layout.hip -- development probe: operand / result lane layout of
// v_mfma_f64_4x4x4f64 (4 blocks) on gfx950.  For each one-hot A lane (B all ones) and each
// one-hot B lane (A all ones) prints the 64-bit mask of result lanes that become nonzero, and
// for pairs (A lane a, B lane b) whether they meet in a product (same block and k).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void probe(int mode, int sel, int sel2, double* out) {
  const int l = threadIdx.x;
  double a, b;
  if (mode == 0) { a = (l == sel) ? 1.0 : 0.0; b = 1.0; }
  else if (mode == 1) { a = 1.0; b = (l == sel) ? 1.0 : 0.0; }
  else { a = (l == sel) ? 1.0 : 0.0; b = (l == sel2) ? 1.0 : 0.0; }
  double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  out[l] = d;
}
int main() {
  double* d; hipMalloc(&d, 64 * sizeof(double));
  double h[64];
  for (int mode = 0; mode < 2; ++mode)
    for (int s = 0; s < 64; ++s) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, mode, s, 0, d);
      hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
      unsigned long long m = 0;
      for (int i = 0; i < 64; ++i) if (h[i] != 0.0) m |= 1ull << i;
      printf("%s lane %2d -> D mask %016llx\n", mode ? "B" : "A", s, m);
    }
  // which (A lane, B lane) pairs multiply: for A lane a, list B lanes b that produce a nonzero D
  for (int a = 0; a < 16; ++a) {
    printf("A lane %2d pairs with B lanes:", a);
    for (int b = 0; b < 64; ++b) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, 2, a, b, d);
      hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
      int hit = -1;
      for (int i = 0; i < 64; ++i) if (h[i] != 0.0) hit = i;
      if (hit >= 0) printf(" %d(D%d)", b, hit);
    }
    printf("\n");
  }
  return 0;
}
