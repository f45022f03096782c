// kernels.hip -- gfx950 (MI355X) kernels of the sparkGLM fitting engine.
//
// K1+K2 fused IRLS pass (irls_pass_kernel<P16>): one streaming pass over the HBM-resident
// design X per IRLS iteration.  Per row block of RB=32 rows:
//   1. LDS-DMA (global_load_lds_dwordx4) of the block's 32 x (16*P16) tile and its y/m/
//      offset/prior values, double-buffered one block ahead;
//   2. eta = X beta + offset (etaCreate, GLM.scala:321-332), inverse link, variance,
//      working weight w and response z (zwCreateBinomial, GLM.scala:359-395) and the
//      deviance / Pearson / loglik partial sums (GLM.scala:90-170) -- rowmath.hpp;
//   3. the weighted Gramian X'WX (lower-triangular 16x16 tiles) on fp64 MFMA
//      (v_mfma_f64_16x16x4_f64) with the accumulators resident in registers for the
//      whole launch, and X'Wz on the VALU (partitionComponents, utils.scala:84-92).
// Each workgroup streams a contiguous range of row blocks (split-K over rows) and writes
// one partial; reduce_partials_kernel sums the partials in a fixed order (deterministic)
// into the packed wire format (lower-triangular X'WX row-major | X'Wz | scalars).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "common.hpp"
#include "kernels.hpp"
#include "procx.hpp"
#include "rowmath.hpp"

#include "fused.hpp"

namespace sglm {

// ---------------------------------------------------------------------------------
// Fixed-order reduction of the workgroup partials into the packed wire format.
// A 256-thread block covers RED_EL consecutive output elements with RED_SEG threads each: thread
// (segment s, element e) sums partials [s n / RED_SEG, (s+1) n / RED_SEG) left to right, then
// segment 0's thread adds the RED_SEG segment sums in segment order -- a fixed two-level order,
// deterministic, and RED_SEG times the threads of one dependent load-add chain per element (a
// p = 20 LM Gram has 238 outputs: one chain over all partials each was a latency-bound 15 us).
// The scalars (deviance, ...) are Neumaier-compensated at both levels.
// ---------------------------------------------------------------------------------
constexpr int RED_SEG = 8, RED_EL = 256 / RED_SEG, RED_BATCH = 32;

__global__ void __launch_bounds__(256) reduce_partials_kernel(const double* __restrict__ part, int64_t stride,
                                                              int nparts, int p, int P16, double* __restrict__ out,
                                                              int extra) {
  // partial layout: T tiles of 256 | X'Wz [16*P16] | NS scalars | extra (the LM Gram's X'1, narrow LMX)
  __shared__ double ss[RED_SEG][RED_EL], cs[RED_SEG][RED_EL];
  const int64_t tri = (int64_t)p * (p + 1) / 2;
  const int64_t total = tri + p + NS + extra;
  const int T = P16 * (P16 + 1) / 2;
  const int el = threadIdx.x % RED_EL, sg = threadIdx.x / RED_EL;
  const int g0 = (int)((int64_t)nparts * sg / RED_SEG), g1 = (int)((int64_t)nparts * (sg + 1) / RED_SEG);
  for (int64_t base = (int64_t)blockIdx.x * RED_EL; base < total; base += (int64_t)gridDim.x * RED_EL) {
    const int64_t e = base + el;
    double s = 0.0, c = 0.0;
    const bool scal = e >= tri + p && e < tri + p + NS;
    if (e < total) {
      int64_t src;
      if (e < tri) {
        int64_t i = (int64_t)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
        while (i * (i + 1) / 2 > e) --i;
        while ((i + 1) * (i + 2) / 2 <= e) ++i;
        const int64_t j = e - i * (i + 1) / 2;
        const int64_t bi = i >> 4, bj = j >> 4;
        const int64_t t = bi * (bi + 1) / 2 + bj;
        src = t * 256 + (i & 15) * 16 + (j & 15);
      } else if (e < tri + p) {
        src = (int64_t)T * 256 + (e - tri);
      } else if (e < tri + p + NS) {
        src = (int64_t)T * 256 + 16 * P16 + (e - tri - p);
      } else {
        src = (int64_t)T * 256 + 16 * P16 + NS + (e - tri - p - NS);
      }
      // the segment's partials left to right, RED_BATCH loads in flight per thread (a 256-partial
      // reduce is one batch: one load latency, not four)
      const double* q = part + src;
      int g = g0;
      if (!scal) {
        for (; g + RED_BATCH <= g1; g += RED_BATCH) {
          double v[RED_BATCH];
#pragma unroll
          for (int u = 0; u < RED_BATCH; ++u) v[u] = q[(int64_t)(g + u) * stride];
#pragma unroll
          for (int u = 0; u < RED_BATCH; ++u) s += v[u];
        }
        for (; g < g1; ++g) s += q[(int64_t)g * stride];
      } else {  // deviance and the other scalars: compensated, in the same order
        for (; g + RED_BATCH <= g1; g += RED_BATCH) {
          double v[RED_BATCH];
#pragma unroll
          for (int u = 0; u < RED_BATCH; ++u) v[u] = q[(int64_t)(g + u) * stride];
#pragma unroll
          for (int u = 0; u < RED_BATCH; ++u) neumaier_add(s, c, v[u]);
        }
        for (; g < g1; ++g) neumaier_add(s, c, q[(int64_t)g * stride]);
      }
    }
    ss[sg][el] = s;
    cs[sg][el] = c;
    __syncthreads();
    if (sg == 0 && e < total) {
      double t = ss[0][el], tc = cs[0][el];
      for (int k = 1; k < RED_SEG; ++k) {
        if (scal) {
          neumaier_add(t, tc, ss[k][el]);
          tc += cs[k][el];
        } else {
          t += ss[k][el];
        }
      }
      out[e] = scal ? t + tc : t;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------
// eta = X beta (+ offset): LM.predict (LM.scala:39-61) / etaCreate.
// ---------------------------------------------------------------------------------
__global__ void predict_kernel(const double* __restrict__ X, int64_t ld, int p, int64_t n,
                               const double* __restrict__ beta, const double* __restrict__ off,
                               double* __restrict__ out, ProcX g) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    if (g.on)
      for (int j = 0; j < p; ++j) s += proc_x(g, i, j) * beta[j];
    else
      for (int j = 0; j < p; ++j) s += X[(int64_t)j * ld + i] * beta[j];
    out[i] = off ? s + off[i] : s;
  }
}

// mu = unlink(eta, m) in place: muCreate (GLM.scala:334-355) / R's family linkinv, the
// response-scale prediction.  One instantiation per family/link.
template <int FAM, int LNK>
__global__ void unlink_kernel(double* __restrict__ v, const double* __restrict__ m, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    v[i] = unlink_fn(FAM, LNK, v[i], m ? m[i] : 1.0);
}

// Block partial sums of y (GLM.scala:420-423 ySums) -- fixed order per block.
__global__ void ysum_kernel(const double* __restrict__ y, int64_t n, double* __restrict__ part) {
  __shared__ double red[4];
  double s = 0.0;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t a = per * blockIdx.x, b = (a + per < n) ? a + per : n;
  for (int64_t i = a + threadIdx.x; i < b; i += blockDim.x) s += y[i];
  for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

// Final-statistics pass over the resident vectors and the last pass's eta: one partial
// of NS scalars per block, summed in a fixed order on the host side reduction.
// One instantiation per family/link (as the pass kernels): an all-families kernel carried every
// family's libm code (lgamma, erfinv, ...) at 438 VGPRs, one wave per SIMD, latency-bound.
// PM > 0 (LM residuals on a resident shard, p <= PM, PM a multiple of 8): the row's p loads of X are
// issued together -- every column slot loads (slots past p re-read column 0, a cache hit) and the
// products enter eta branch-free -- where the runtime-p loop waited for each load before its fma
// (configs[0]: 34 us for a 168 MB pass, one HBM latency per column).  The same fma chain, so the
// same eta.
template <int FAM, int LNK, int PM = 0>
__global__ void __launch_bounds__(256) stats_kernel(StatsArgs a) {
  __shared__ double red[4][NS];
  RowAcc acc;
#pragma unroll
  for (int k = 0; k < NS; ++k) acc.s[k] = 0.0;
  const int64_t per = (a.n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = per * blockIdx.x, hi = (lo + per < a.n) ? lo + per : a.n;
  const double ybar = a.ybar_dev ? *a.ybar_dev : a.ybar;
  double bl[PM > 0 ? PM : 1];
  if constexpr (PM > 0) {
#pragma unroll
    for (int j = 0; j < PM; ++j)
      bl[j] = j >= a.p ? 0.0 : a.beta_by_value ? a.bv[j < STATS_BETA_MAX ? j : 0] : a.beta[j];
  }
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const double m = a.m ? a.m[i] : 1.0;
    const double pw = a.prior ? a.prior[i] : 1.0;
    double eta = 0.0;
    if constexpr (PM > 0) {
      double x[PM];
#pragma unroll
      for (int j = 0; j < PM; ++j) x[j] = a.X[(int64_t)(j < a.p ? j : 0) * a.ld + i];
#pragma unroll
      for (int j = 0; j < PM; ++j) eta = j < a.p ? fma(x[j], bl[j], eta) : eta;
    } else if (a.X) {  // LM residuals: X*coefs in predict_kernel's order (LM.scala:173-174)
      if (a.beta_by_value)
        for (int j = 0; j < a.p; ++j) eta += a.X[(int64_t)j * a.ld + i] * a.bv[j];
      else
        for (int j = 0; j < a.p; ++j) eta += a.X[(int64_t)j * a.ld + i] * a.beta[j];
    } else if (a.eta) {
      eta = a.eta[i];
    }
    stats_row(FAM, LNK, a.mode, eta, a.y[i], m, pw, a.mu0, ybar, a.m != nullptr, acc);
  }
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    double v = acc.s[k];
    for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < NS) {
    const int k = threadIdx.x;
    a.partials[(int64_t)blockIdx.x * NS + k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
  }
}

// LM.fit's p x p solve on the device (engine.cpp lm_device; p <= 64): the host solver's Cholesky
// (solve.cpp chol_factor + chol_solve), element for element in the same operation order without
// contraction, so the coefficients come out bitwise the host's (driver.cpp lm_drive checks that and
// otherwise reruns the residual pass at its own).  One wave; lane i holds row i of the matrix in
// registers (a[j] = A(i, j), PM = p rounded up to 4 / 8, every loop unrolled, no branch): step k reads
// the pivot from lane k, scales column k (L(i, k) = A(i, k) / sqrt(d) as 1 / sqrt(d) times, the host's
// order) and subtracts L(i, k) L(j, k) from A(i, j), j > k, with L(j, k) read from lane j -- each
// element receives its subtractions in ascending k, chol_factor's left-looking order, and L(j, k) == 0
// skips the subtraction as there.  The forward sweep L t = b runs in the same steps, the back
// substitution L' x = t as a column sweep over L staged once in LDS (the host chol_solve's order).
// Rows p..PM-1 are identity padding: their steps divide by 1 and subtract zeros, which leaves the real
// rows' values unchanged (their t stays 0 and the back substitution skips them), so the whole
// factorization is one basic block the compiler can overlap
// across steps.  A pivot that is not positive and finite sets the failure flag (the host stops there;
// the values past it are not used).  Earlier forms -- one wave in LDS, left-looking, 37 us at p = 20;
// right-looking 26 us; four waves over LDS with a barrier a step 19 us -- were bound by the per-step
// LDS round trips and barriers on the 20-pivot chain.
// Out: beta[p] (NaN when a pivot failed); aux[0] = sum y / rows (LM.scala:167-168), aux[1] = 1 where
// the host would leave Cholesky (a non-positive pivot, or the pivot ratio below LU_SWITCH_RATIO:
// solve.cpp chol_pivot_ratio).
__device__ __forceinline__ double lane_bcast(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
//
// One pass (LmOnePass, the LM Gram pass ran with PassArgs::lm_extras): the residual statistics of
// LM.scala:160-188 from the Gram pass's sums instead of a second pass over X --
//   SSE = y'y - 2 b'X'y + b'X'X b,  top = b'X'X b - 2 ybar b'X'1 + n ybar^2,  bot = y'y - 2 ybar sum y + n ybar^2
// (sum (y - Xb)^2, sum (Xb - ybar)^2, sum (y - ybar)^2 expanded).  Each is a difference of sums up to
// max(y'y, b'X'X b, n ybar^2), so its rounding relative to the result grows with that ratio: above
// LM_ONEPASS_MAX_RATIO (or with any of the three <= 0, e.g. an intercept-only model's top = 0) the
// statistics are flagged (S_BAD = 1) and lm_drive reruns the residual pass, the reference's own form.
// The fit's whole result buffer -- packed | X'1 | statistics | b -- is written to pinned host memory
// (no copy blit, one synchronisation): the inputs copied, the statistics and b from registers.
template <int PM>
__global__ void __launch_bounds__(64) lm_chol_kernel(const double* __restrict__ packed, int p, double ratio_min,
                                                     double* __restrict__ beta, double* __restrict__ aux,
                                                     LmOnePass op) {
#pragma clang fp contract(off)
  constexpr int LDL = PM + 1;
  __shared__ double Ls[PM * LDL];  // L(r, c) at Ls[r LDL + c] for the back substitution
  __shared__ double bs[PM];        // one pass: b for every lane
  const int i = threadIdx.x;
  const bool row = i < p;
  const int64_t tri = (int64_t)p * (p + 1) / 2;
  double a[PM];
#pragma unroll
  for (int j = 0; j < PM; ++j) {  // unpack_gram's lower triangle: A(i, j) = packed[i (i + 1) / 2 + j], j <= i
    const bool in = row && j <= i;  // every lane loads (index 0 outside): no branch around the loads
    const double v = packed[in ? (int64_t)i * (i + 1) / 2 + j : 0];
    a[j] = in ? v : (i == j ? 1.0 : 0.0);
  }
  const double dgi = row ? packed[(int64_t)i * (i + 1) / 2 + i] : 0.0;
  double ti = row ? packed[tri + i] : 0.0;
  double diag = 1.0;
  bool fail = false;
#pragma unroll
  for (int k = 0; k < PM; ++k) {
    const double d = lane_bcast(a[k], k);
    fail = fail || !(d > 0.0) || !isfinite(d);
    const double sq = sqrt(d);
    double inv = 1.0 / sq;
    asm volatile("" : "+v"(inv));  // formed on every lane, not in a branch around lane k (a step stays one block)
    const double lik = (i == k) ? sq : a[k] * inv;  // L(i, k), lanes i >= k
    const double tk = lane_bcast(ti / sq, k);      // L t = b: t_k /= L(k, k); t_i -= L(i, k) t_k, i > k
    if (i > k && row) ti -= lik * tk;
    if (i == k) ti = tk;
#pragma unroll
    for (int j = k + 1; j < PM; ++j) {
      const double l = lane_bcast(lik, j);
      const double nv = a[j] - lik * l;
      a[j] = (i >= j && l != 0.0) ? nv : a[j];
    }
    if (i >= k) a[k] = lik;
    if (i == k) diag = sq;
  }
  if (!fail) {
    if (i < PM) {
#pragma unroll
      for (int j = 0; j < PM; ++j) Ls[i * LDL + j] = a[j];
    }
    __syncthreads();
    double tb = ti;
#pragma unroll
    for (int r = PM - 1; r >= 0; --r) {  // L' x = t: x_r = t_r / L(r, r); t_i -= L(r, i) x_r, i < r
      const double xr = lane_bcast(tb / diag, r);
      const double lri = Ls[r * LDL + (i < PM ? i : 0)];
      tb = (i < r && r < p) ? tb - lri * xr : tb;  // padding rows stay out
      if (i == r) tb = xr;
    }
    if (row) beta[i] = tb;
    if (row && op.host) op.host[(beta - packed) + i] = tb;
    if (op.stats) {  // the residual statistics from the Gram pass's sums (one pass)
      if (i < PM) bs[i] = row ? tb : 0.0;
      __syncthreads();
      double ab = 0.0;  // (X'X b)_i, j ascending
      if (row) {
        for (int j = 0; j < p; ++j) {
          const int64_t idx = j <= i ? (int64_t)i * (i + 1) / 2 + j : (int64_t)j * (j + 1) / 2 + i;
          ab += packed[idx] * bs[j];
        }
      }
      double q = row ? tb * ab : 0.0, bxy = row ? tb * packed[tri + i] : 0.0, bx1 = row ? tb * op.x1[i] : 0.0;
      for (int o = 1; o < 64; o <<= 1) {  // butterfly sums: every lane holds the same totals
        q += __shfl_xor(q, o);
        bxy += __shfl_xor(bxy, o);
        bx1 += __shfl_xor(bx1, o);
      }
      if (i == 0) {
        const double yy = packed[tri + p + S_PEARSON], ys = packed[tri + p + S_DEV], nr = packed[tri + p + S_SUMW];
        const double yb = ys / nr, nyb2 = nr * yb * yb;
        const double sse = (yy - 2.0 * bxy) + q;
        const double top = (q - 2.0 * yb * bx1) + nyb2;
        const double bot = (yy - 2.0 * yb * ys) + nyb2;
        const double big = fmax(yy, fmax(q, nyb2)), small = fmin(sse, fmin(top, bot));
        const bool ok = small > 0.0 && big < LM_ONEPASS_MAX_RATIO * small && isfinite(big);
        double sv[NS];
        for (int k = 0; k < NS; ++k) sv[k] = 0.0;
        sv[S_DEV] = sse;
        sv[S_PEARSON] = top;
        sv[S_LL] = bot;
        sv[S_SUMW] = nr;
        sv[S_BAD] = ok ? 0.0 : 1.0;
        for (int k = 0; k < NS; ++k) {
          op.stats[k] = sv[k];
          if (op.host) op.host[(op.stats - packed) + k] = sv[k];
        }
      }
    }
  } else {
    if (row) beta[i] = __builtin_nan("");  // no coefficients: the host sees NaN and runs its own residual pass
    if (row && op.host) op.host[(beta - packed) + i] = __builtin_nan("");
    if (op.stats && i == 0) {
      for (int k = 0; k < NS; ++k) {
        op.stats[k] = k == S_BAD ? 1.0 : 0.0;
        if (op.host) op.host[(op.stats - packed) + k] = k == S_BAD ? 1.0 : 0.0;
      }
    }
  }
  double r = (row && dgi > 0.0) ? (diag * diag) / dgi : 1.0;  // chol_pivot_ratio: min over j (exact, any order)
  for (int o = 1; o < 64; o <<= 1) r = fmin(r, __shfl_xor(r, o));
  if (i == 0) {
    aux[0] = packed[tri + p + S_DEV] / packed[tri + p + S_SUMW];
    aux[1] = (fail || fmin(1.0, r) < ratio_min) ? 1.0 : 0.0;
  }
  if (op.host)  // the rest of the result buffer: the kernel's inputs packed | X'1, [0, ncopy)
    for (int64_t k = i; k < op.ncopy; k += 64) op.host[k] = packed[k];
}

// The stats partials [nparts][NS] summed on the device into out[NS] (no D2H of the partials):
// thread (segment s, scalar k) sums partials [s n / 32, (s+1) n / 32) in order, Neumaier-compensated,
// then thread k adds the 32 segment sums and their compensations in segment order.
// host != null (the LM device round trip): the kernel also writes the fit's result buffer into pinned
// host memory -- src[0, ncopy) with out at src + out_off -- so no copy blit follows it (~4 us).
__global__ void __launch_bounds__(256) reduce_stats_kernel(const double* __restrict__ part, int nparts,
                                                           double* __restrict__ out, const double* __restrict__ src,
                                                           double* __restrict__ host, int64_t ncopy, int64_t out_off) {
  __shared__ double ss[32][NS], cs[32][NS];
  const int k = threadIdx.x % NS, sg = threadIdx.x / NS;
  const int g0 = (int)((int64_t)nparts * sg / 32), g1 = (int)((int64_t)nparts * (sg + 1) / 32);
  double s = 0.0, c = 0.0;
  int g = g0;
  for (; g + RED_BATCH <= g1; g += RED_BATCH) {  // RED_BATCH loads in flight ahead of the ordered compensated adds
    double v[RED_BATCH];
#pragma unroll
    for (int u = 0; u < RED_BATCH; ++u) v[u] = part[(int64_t)(g + u) * NS + k];
#pragma unroll
    for (int u = 0; u < RED_BATCH; ++u) neumaier_add(s, c, v[u]);
  }
  for (; g < g1; ++g) neumaier_add(s, c, part[(int64_t)g * NS + k]);
  ss[sg][k] = s;
  cs[sg][k] = c;
  __syncthreads();
  if (threadIdx.x < NS) {
    double t = 0.0, tc = 0.0;
    for (int q = 0; q < 32; ++q) {
      neumaier_add(t, tc, ss[q][threadIdx.x]);
      tc += cs[q][threadIdx.x];
    }
    out[threadIdx.x] = t + tc;
    if (host) host[out_off + threadIdx.x] = t + tc;
  }
  if (host)
    for (int64_t e = threadIdx.x; e < ncopy; e += blockDim.x)
      if (e < out_off || e >= out_off + NS) host[e] = src[e];
}

// ---------------------------------------------------------------------------------
// Seeded synthetic design (bit-identical to sparkglm_amd/synth.py; no FMA contraction).
// ---------------------------------------------------------------------------------
__global__ void synth_kernel(int kind, int64_t row0, int64_t n, int p, uint64_t seed, double scale, double* X,
                             int64_t ld, double* y, double* m, double* off, double* prior) {
#pragma clang fp contract(off)
  const uint64_t kx = splitmix64(seed), ky = splitmix64(seed ^ 0x5555555555555555ull),
                 ko = splitmix64(seed ^ 0x3333333333333333ull), kp = splitmix64(seed ^ 0x0F0F0F0F0F0F0F0Full);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t gi = (uint64_t)(row0 + i);
    double eta = 0.0;
    for (int j = 0; j < p; ++j) {
      const double x = gen_x(kind, kx, gi, p, j, scale);  // kind 3: positive design (eta > 0)
      if (X) X[(int64_t)j * ld + i] = x;                  // procedural shards keep only y
      double bj;
      if (kind == 3) bj = (j == 0) ? 1.0 : 0.1 * (double)((j % 5) + 1);
      else bj = (j == 0) ? -0.25 : 0.5 * (double)((j % 5) - 2);
      const double prod = x * bj;
      eta = eta + prod;
    }
    const double u = unif(ky + gi);
    if (kind == 0) {
      double pr = 0.5 + 0.25 * eta;
      pr = pr < 0.02 ? 0.02 : (pr > 0.98 ? 0.98 : pr);
      y[i] = u < pr ? 1.0 : 0.0;
    } else if (kind == 1) {
      y[i] = eta + (2.0 * u - 1.0);
    } else if (kind == 3) {
      y[i] = (0.25 + 1.5 * u) / eta;  // mean 1/eta (gamma / inverse link), y > 0
    } else {
      double lam = 1.0 + 0.5 * eta;
      lam = lam < 0.1 ? 0.1 : lam;
      y[i] = floor(u * 2.0 * lam);
      if (off) off[i] = (2.0 * unif(ko + gi) - 1.0) * 0.1;
      if (prior) prior[i] = 0.5 + unif(kp + gi);
    }
    if (m) m[i] = 1.0;
  }
}

// ---------------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------------
// Kernel variants: P16 = ceil(p / 16) column blocks of 16 in 2..16 (p <= 256).  K1 is built for
// even P16 (NW = P16/2 waves, two tile rows each); K1r for every P16 >= 5.  An odd count runs K1r
// when the pass may (pass_uses_split) and is rounded up to K1's even count otherwise -- so p = 240
// runs 120 tiles of 16 x 16 per k-step instead of 136.
// K1r runs P16 >= the threshold PassArgs::fused_split carries (1: the default, K1R_MIN_P16 for even
// counts and K1R_MIN_ODD for odd ones; 0: never) -- one 12-wave workgroup per CU; K1 the rest.
// Same-box A/B (profiles/r04_midp_ab.txt): p = 240 K1r<15> 10.39 ms against K1r<16> 10.91 and K1<16>
// 11.55; but p = 80 K1r<5> 10.25 against K1<6> at three workgroups per CU 9.87, p = 112 K1r<7> 10.37
// against K1<8> 9.78-10.33 -- below P16 = 9 the eight Gram waves carry two to three tiles each.
// Its DMA addresses the 4 columns of a quad by 32-bit lane offsets (3 ld + 32 rows, in bytes),
// which bounds the shard at ~178M rows.
constexpr int K1R_MIN_P16 = 10, K1R_MIN_ODD = 9;
// K1 runs the odd counts 5 and 7 itself (its tiles are runs of the tile sequence, not row pairs:
// p = 65..80 and 97..112 run 15 / 28 tiles instead of 21 / 36); above, an odd count K1r may not run
// rounds up to K1's even one.
constexpr int K1_MAX_ODD = 7;
bool pass_uses_split(int P16, int fused_split, int64_t ld) {
  const int thr = fused_split == 1 ? ((P16 & 1) ? K1R_MIN_ODD : K1R_MIN_P16) : fused_split;
  return fused_split != 0 && P16 >= 5 && P16 >= thr && ld * 24 + 4096 < ((int64_t)1 << 32);
}
int pass_variant(int p, int fused_split, int64_t ld) {
  int P16 = (p + 15) / 16;
  if ((P16 & 1) && P16 > K1_MAX_ODD && !pass_uses_split(P16, fused_split, ld)) ++P16;
  return P16 < 2 ? 2 : P16;
}
int pass_stride(int P16) { return (P16 * (P16 + 1) / 2) * 256 + 16 * P16 + NS; }

template <int P16>
static int wg_per_cu_t() { return Geo<P16>::WG_PER_CU; }

// K1's workgroups per CU (even P16; K1r runs one workgroup per CU)
int pass_wg_per_cu(int P16) {
  switch (P16) {
    case 2: return wg_per_cu_t<2>();
    case 4: return wg_per_cu_t<4>();
    case 5: return wg_per_cu_t<5>();
    case 6: return wg_per_cu_t<6>();
    case 7: return wg_per_cu_t<7>();
    case 8: return wg_per_cu_t<8>();
    case 10: return wg_per_cu_t<10>();
    case 12: return wg_per_cu_t<12>();
    case 14: return wg_per_cu_t<14>();
    default: return wg_per_cu_t<16>();
  }
}

template <int P16>
static hipError_t launch_pass_p(const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  if constexpr (P16 >= 6)
    if (pass_uses_split(P16, a.fused_split, a.ld)) return launch_pass_r_fl<P16>(a, grid, st, e0, e1);
  return launch_pass_k1<P16>(a, grid, st, e0, e1);
}

hipError_t launch_pass(int P16, const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  if ((P16 & 1) && P16 >= 5) return launch_pass_odd(P16, a, grid, st, e0, e1);  // fused_odd.hip
  switch (P16) {
    case 2: return launch_pass_p<2>(a, grid, st, e0, e1);
    case 4: return launch_pass_p<4>(a, grid, st, e0, e1);
    case 6: return launch_pass_p<6>(a, grid, st, e0, e1);
    case 8: return launch_pass_p<8>(a, grid, st, e0, e1);
    case 10: return launch_pass_p<10>(a, grid, st, e0, e1);
    case 12: return launch_pass_p<12>(a, grid, st, e0, e1);
    case 14: return launch_pass_p<14>(a, grid, st, e0, e1);
    case 16: return launch_pass_p<16>(a, grid, st, e0, e1);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_lm_chol(const double* packed, int p, double ratio_min, double* beta, double* aux, hipStream_t st,
                          const LmOnePass& op) {
  if (p < 1 || p > 64) return hipErrorInvalidValue;
  // PM = p rounded up to 4 up to 32, to 8 above (identity padding: a padding step costs what a real one does)
  const int pm = p <= 32 ? (p + 3) / 4 * 4 : (p + 7) / 8 * 8;
  switch (pm) {
#define SGLM_CHOL_CASE(PM) \
  case PM: hipLaunchKernelGGL(lm_chol_kernel<PM>, dim3(1), dim3(64), 0, st, packed, p, ratio_min, beta, aux, op); break;
    SGLM_CHOL_CASE(4) SGLM_CHOL_CASE(8) SGLM_CHOL_CASE(12) SGLM_CHOL_CASE(16) SGLM_CHOL_CASE(20) SGLM_CHOL_CASE(24)
    SGLM_CHOL_CASE(28) SGLM_CHOL_CASE(32) SGLM_CHOL_CASE(40) SGLM_CHOL_CASE(48) SGLM_CHOL_CASE(56) SGLM_CHOL_CASE(64)
#undef SGLM_CHOL_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_reduce_stats(const double* part, int nparts, double* out, hipStream_t st, const double* src,
                               double* host, int64_t ncopy) {
  // out's offset inside src: only meaningful (and only computed) when the result buffer is copied
  const int64_t out_off = (src && host) ? (int64_t)(out - src) : 0;
  hipLaunchKernelGGL(reduce_stats_kernel, dim3(1), dim3(32 * NS), 0, st, part, nparts, out, src, host, ncopy, out_off);
  return hipGetLastError();
}

hipError_t launch_stats(const StatsArgs& a, int grid, hipStream_t st) {
  const dim3 gr(grid), bl(256);
  if (a.X && a.mode == MODE_LM_RESID && a.p >= 1 && a.p <= 64) {  // the LM residual pass, loads together
    switch ((a.p + 7) / 8) {
      case 1: hipLaunchKernelGGL((stats_kernel<FAM_GAUSSIAN, LNK_IDENTITY, 8>), gr, bl, 0, st, a); break;
      case 2: hipLaunchKernelGGL((stats_kernel<FAM_GAUSSIAN, LNK_IDENTITY, 16>), gr, bl, 0, st, a); break;
      case 3: hipLaunchKernelGGL((stats_kernel<FAM_GAUSSIAN, LNK_IDENTITY, 24>), gr, bl, 0, st, a); break;
      case 4: hipLaunchKernelGGL((stats_kernel<FAM_GAUSSIAN, LNK_IDENTITY, 32>), gr, bl, 0, st, a); break;
      case 5: hipLaunchKernelGGL((stats_kernel<FAM_GAUSSIAN, LNK_IDENTITY, 40>), gr, bl, 0, st, a); break;
      case 6: hipLaunchKernelGGL((stats_kernel<FAM_GAUSSIAN, LNK_IDENTITY, 48>), gr, bl, 0, st, a); break;
      case 7: hipLaunchKernelGGL((stats_kernel<FAM_GAUSSIAN, LNK_IDENTITY, 56>), gr, bl, 0, st, a); break;
      default: hipLaunchKernelGGL((stats_kernel<FAM_GAUSSIAN, LNK_IDENTITY, 64>), gr, bl, 0, st, a); break;
    }
  } else if (a.mode == MODE_LM_RESID || (a.family == FAM_GAUSSIAN && a.link == LNK_IDENTITY))
    hipLaunchKernelGGL((stats_kernel<FAM_GAUSSIAN, LNK_IDENTITY>), gr, bl, 0, st, a);
  else if (a.family == FAM_BINOMIAL && a.link == LNK_LOGIT)
    hipLaunchKernelGGL((stats_kernel<FAM_BINOMIAL, LNK_LOGIT>), gr, bl, 0, st, a);
  else if (a.family == FAM_BINOMIAL && a.link == LNK_PROBIT)
    hipLaunchKernelGGL((stats_kernel<FAM_BINOMIAL, LNK_PROBIT>), gr, bl, 0, st, a);
  else if (a.family == FAM_BINOMIAL && a.link == LNK_CLOGLOG)
    hipLaunchKernelGGL((stats_kernel<FAM_BINOMIAL, LNK_CLOGLOG>), gr, bl, 0, st, a);
  else if (a.family == FAM_POISSON && a.link == LNK_LOG)
    hipLaunchKernelGGL((stats_kernel<FAM_POISSON, LNK_LOG>), gr, bl, 0, st, a);
  else if (a.family == FAM_GAMMA && a.link == LNK_INVERSE)
    hipLaunchKernelGGL((stats_kernel<FAM_GAMMA, LNK_INVERSE>), gr, bl, 0, st, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_reduce(const double* part, int64_t stride, int nparts, int p, int P16, double* out, hipStream_t st,
                         hipEvent_t e1, int extra) {
  const int64_t total = (int64_t)p * (p + 1) / 2 + p + NS + extra;
  int blocks = (int)((total + RED_EL - 1) / RED_EL);
  if (blocks > 8192) blocks = 8192;
  hipExtLaunchKernelGGL(reduce_partials_kernel, dim3(blocks), dim3(256), 0, st, nullptr, e1, 0, part, stride, nparts, p, P16,
                        out, extra);
  return hipGetLastError();
}

hipError_t launch_predict(const double* X, int64_t ld, int p, int64_t n, const double* beta, const double* off,
                          double* out, hipStream_t st, const ProcX& g) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(predict_kernel, dim3((unsigned)blocks), dim3(256), 0, st, X, ld, p, n, beta, off, out, g);
  return hipGetLastError();
}

hipError_t launch_unlink(double* v, const double* m, int64_t n, int family, int link, hipStream_t st) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks < 1) blocks = 1;
  const dim3 g((unsigned)blocks), b(256);
  if (family == FAM_BINOMIAL && link == LNK_LOGIT)
    hipLaunchKernelGGL((unlink_kernel<FAM_BINOMIAL, LNK_LOGIT>), g, b, 0, st, v, m, n);
  else if (family == FAM_BINOMIAL && link == LNK_PROBIT)
    hipLaunchKernelGGL((unlink_kernel<FAM_BINOMIAL, LNK_PROBIT>), g, b, 0, st, v, m, n);
  else if (family == FAM_BINOMIAL && link == LNK_CLOGLOG)
    hipLaunchKernelGGL((unlink_kernel<FAM_BINOMIAL, LNK_CLOGLOG>), g, b, 0, st, v, m, n);
  else if (family == FAM_GAUSSIAN)
    return hipSuccess;  // identity
  else if (family == FAM_POISSON)
    hipLaunchKernelGGL((unlink_kernel<FAM_POISSON, LNK_LOG>), g, b, 0, st, v, m, n);
  else if (family == FAM_GAMMA)
    hipLaunchKernelGGL((unlink_kernel<FAM_GAMMA, LNK_INVERSE>), g, b, 0, st, v, m, n);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_ysum(const double* y, int64_t n, double* part, int nparts, hipStream_t st) {
  hipLaunchKernelGGL(ysum_kernel, dim3(nparts), dim3(256), 0, st, y, n, part);
  return hipGetLastError();
}

uint64_t splitmix64_host(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

hipError_t launch_synth(int kind, int64_t row0, int64_t n, int p, uint64_t seed, double scale, double* X, int64_t ld,
                        double* y, double* m, double* off, double* prior, hipStream_t st) {
  int64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, st, kind, row0, n, p, seed, scale, X, ld, y,
                     m, off, prior);
  return hipGetLastError();
}

}  // namespace sglm
