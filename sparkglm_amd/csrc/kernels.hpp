// kernels.hpp -- host-side launchers of the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace sglm {

// column-block count P16 of the fused kernel a pass over p columns runs (odd: K1r only)
int pass_variant(int p, int fused_split, int64_t ld);
int pass_stride(int P16);       // doubles per workgroup partial
int pass_wg_per_cu(int P16);    // workgroups per CU the variant is built for
bool pass_uses_split(int P16, int fused_split, int64_t ld);  // K1r (one 12-wave workgroup per CU) for this pass
// e0 / e1: HIP events the launch itself records at the kernel's start / end (hipExtLaunchKernel: no
// marker packets between the kernels of a pass; null = none)
hipError_t launch_pass(int P16, const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0 = nullptr,
                       hipEvent_t e1 = nullptr);
hipError_t launch_pass_odd(int P16, const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1);  // fused_odd.hip: K1r, P16 5..15 odd
hipError_t launch_stats(const StatsArgs& a, int grid, hipStream_t st);
// [nparts][NS] -> [NS]; host != null: also src[0, ncopy) (out inside it) into host memory the device can write
hipError_t launch_reduce_stats(const double* part, int nparts, double* out, hipStream_t st, const double* src = nullptr,
                               double* host = nullptr, int64_t ncopy = 0);
// LM.fit's solve on the device, bitwise the host Cholesky (p <= 64): beta[p], aux = {ybar, leave-Cholesky flag}.
// One pass (op.stats set; the Gram pass ran with PassArgs::lm_extras): also the residual statistics from
// the Gram pass's sums (x1 = X'1 [p] right after the packed Gram) into op.stats; with op.host the
// result buffer -- packed[0, ncopy) and beta / op.stats (which lie inside the same allocation past it,
// at the same offsets) -- is written to pinned host memory.
struct LmOnePass {
  const double* x1 = nullptr;
  double* stats = nullptr;  // [NS]: SSE, top, bot, rows, S_BAD = 1 when lm_drive must rerun the residual pass
  double* host = nullptr;
  int64_t ncopy = 0;
};
constexpr double LM_ONEPASS_MAX_RATIO = 1e4;  // max(y'y, b'X'Xb, n ybar^2) / min(SSE, top, bot) at most
hipError_t launch_lm_chol(const double* packed, int p, double ratio_min, double* beta, double* aux, hipStream_t st,
                          const LmOnePass& op = LmOnePass{});
// extra: elements past the NS scalars summed too (the LM Gram's X'1, narrow LMX), out[tri + p + NS + k]
hipError_t launch_reduce(const double* part, int64_t stride, int nparts, int p, int P16, double* out, hipStream_t st,
                         hipEvent_t e1 = nullptr, int extra = 0);
hipError_t launch_predict(const double* X, int64_t ld, int p, int64_t n, const double* beta, const double* off,
                          double* out, hipStream_t st, const ProcX& g);
hipError_t launch_unlink(double* v, const double* m, int64_t n, int family, int link, hipStream_t st);
hipError_t launch_ysum(const double* y, int64_t n, double* part, int nparts, hipStream_t st);
uint64_t splitmix64_host(uint64_t x);
hipError_t launch_synth(int kind, int64_t row0, int64_t n, int p, uint64_t seed, double scale, double* X, int64_t ld,
                        double* y, double* m, double* off, double* prior, hipStream_t st);

// narrow path (narrow.hip): p <= 64
int narrow_variant(int p);      // column blocks of 16 (1..4)
int narrow_stride(int P16);     // doubles per workgroup partial (reduce_partials_kernel layout)
int narrow_wg_per_cu();
int narrow_rows_per_wg(int P16); // rows one workgroup streams per block step (waves x rows per block)
hipError_t launch_narrow(int P16, const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0 = nullptr,
                         hipEvent_t e1 = nullptr);

// wide path (wide.hip)
int wide_panels(int p);
int64_t wide_stride();
// ov: the overlapped-chunk variant (wide_rows_ov_kernel: <= 96 VGPRs, fits beside the Gram kernels)
hipError_t launch_wide_rows(const WideRowArgs& a, int grid, hipStream_t st, bool ov = false);
hipError_t launch_proc_gen(const ProcGenArgs& a, int grid, hipStream_t st);
int wide_gram_wg_per_cu(bool diag);
hipError_t launch_wide_gram(const WideGramArgs& a, bool diag, int grid, hipStream_t st);
hipError_t launch_wide_reduce(const double* part, int64_t stride, const int* st_range, int p, const double* rowpart,
                              int nrow, double* out, hipStream_t st);
hipError_t launch_sum_chunks(const double* chunks, int nch, int p, double* out, hipStream_t st);
hipError_t launch_unpack_lower(const double* packed, int p, double* A, double* b, hipStream_t st, bool full = false);
// x = A b, A column-major p x p, summed over k in ascending order (the reference's inv * b)
hipError_t launch_inv_gemv(const double* A, int p, const double* b, double* x, hipStream_t st);

}  // namespace sglm
