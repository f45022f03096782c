// graph_probe.hip -- host overhead of a short fixed kernel sequence: five back-to-back launches +
// stream synchronisation, against the same five captured once into a hipGraph and replayed.
// (Question behind it: would a graph shorten an LM.fit whose kernels sum to ~97 us of a 115 us
// wall?)  Build: hipcc --offload-arch=gfx950 -O2 tools/graph_probe.hip -o build/graph_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));            \
      return 1;                                                             \
    }                                                                       \
  } while (0)

// spin for ~us microseconds of device time (s_memrealtime: 100 MHz)
__global__ void busy(double* out, int us) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  double s = 0.0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)us * 100) s += 1.0;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = s;
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  double* d;
  CHK(hipMalloc(&d, 64));
  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int us[5] = {45, 5, 10, 31, 5};   // the LM fit's kernel durations
  const int grid[5] = {256, 8, 1, 1024, 1};
  auto seq = [&]() {
    for (int k = 0; k < 5; ++k) hipLaunchKernelGGL(busy, dim3(grid[k]), dim3(256), 0, st, d, us[k]);
  };
  for (int w = 0; w < 50; ++w) seq();
  CHK(hipStreamSynchronize(st));
  std::vector<double> a, b;
  for (int it = 0; it < 300; ++it) {
    const auto t0 = std::chrono::steady_clock::now();
    seq();
    CHK(hipStreamSynchronize(st));
    a.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  hipGraph_t g;
  hipGraphExec_t ge;
  CHK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  seq();
  CHK(hipStreamEndCapture(st, &g));
  CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 50; ++w) CHK(hipGraphLaunch(ge, st));
  CHK(hipStreamSynchronize(st));
  for (int it = 0; it < 300; ++it) {
    const auto t0 = std::chrono::steady_clock::now();
    CHK(hipGraphLaunch(ge, st));
    CHK(hipStreamSynchronize(st));
    b.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  std::printf("five launches (device 96 us): stream median %.1f us min %.1f; graph median %.1f us min %.1f\n",
              median(a), *std::min_element(a.begin(), a.end()), median(b), *std::min_element(b.begin(), b.end()));
  // the same 96 us of device time as 1 and as 3 launches: what a fused sequence would save
  for (int nk : {1, 3}) {
    std::vector<double> c;
    const int one[1] = {96}, three[3] = {50, 15, 31};
    for (int it = 0; it < 350; ++it) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int k = 0; k < nk; ++k)
        hipLaunchKernelGGL(busy, dim3(256), dim3(256), 0, st, d, nk == 1 ? one[k] : three[k]);
      CHK(hipStreamSynchronize(st));
      if (it >= 50) c.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::printf("%d launch(es) (device 96 us): stream median %.1f us min %.1f\n", nk, median(c),
                *std::min_element(c.begin(), c.end()));
  }
  CHK(hipGraphExecDestroy(ge));
  CHK(hipGraphDestroy(g));
  CHK(hipStreamDestroy(st));
  CHK(hipFree(d));
  return 0;
}
