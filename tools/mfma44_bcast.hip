// mfma44_bcast.hip -- development probe: v_mfma_f64_4x4x4f64 with CBSZ = 2, ABID = x: does every
// block use block x's A operand?  Prints the max deviation from that model for x = 0..3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
template <int X>
__global__ void k(const double* a, const double* b, double* out) {
  const int l = threadIdx.x;
  out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], 0.0, 2, X, 0);
}
int main() {
  double ha[64], hb[64], hd[64];
  for (int i = 0; i < 64; ++i) { ha[i] = 1.0 + i; hb[i] = 1.0 / (1.0 + i * 0.37); }
  double *a, *b, *d;
  hipMalloc(&a, 512); hipMalloc(&b, 512); hipMalloc(&d, 512);
  hipMemcpy(a, ha, 512, hipMemcpyHostToDevice); hipMemcpy(b, hb, 512, hipMemcpyHostToDevice);
  for (int x = 0; x < 4; ++x) {
    if (x == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, a, b, d);
    if (x == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, a, b, d);
    if (x == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, a, b, d);
    if (x == 3) hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, a, b, d);
    hipMemcpy(hd, d, 512, hipMemcpyDeviceToHost);
    double err = 0;
    for (int dl = 0; dl < 64; ++dl) {
      const int m = dl / 16, blk = (dl % 16) / 4, n = dl % 4;
      double s = 0;
      for (int kk = 0; kk < 4; ++kk) s += ha[16 * kk + 4 * x + m] * hb[16 * kk + 4 * blk + n];
      err = fmax(err, fabs(s - hd[dl]) / fabs(s));
    }
    printf("abid %d: max rel dev from block-%d broadcast model %.3e\n", x, x, err);
  }
  return 0;
}
