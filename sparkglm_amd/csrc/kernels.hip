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
constexpr int RED_SEG = 8, RED_EL = 256 / RED_SEG;

__global__ void __launch_bounds__(256) reduce_partials_kernel(const double* __restrict__ part, int64_t stride,
                                                              int nparts, int p, int P16, double* __restrict__ out) {
  // partial layout: T tiles of 256 | X'Wz [16*P16] | NS scalars
  __shared__ double ss[RED_SEG][RED_EL], cs[RED_SEG][RED_EL];
  const int64_t tri = (int64_t)p * (p + 1) / 2;
  const int64_t total = tri + p + NS;
  const int T = P16 * (P16 + 1) / 2;
  const int el = threadIdx.x % RED_EL, sg = threadIdx.x / RED_EL;
  const int g0 = (int)((int64_t)nparts * sg / RED_SEG), g1 = (int)((int64_t)nparts * (sg + 1) / RED_SEG);
  for (int64_t base = (int64_t)blockIdx.x * RED_EL; base < total; base += (int64_t)gridDim.x * RED_EL) {
    const int64_t e = base + el;
    double s = 0.0, c = 0.0;
    const bool scal = e >= tri + p;
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
      } else {
        src = (int64_t)T * 256 + 16 * P16 + (e - tri - p);
      }
      // the segment's partials left to right, 8 loads in flight per thread
      const double* q = part + src;
      int g = g0;
      if (!scal) {
        for (; g + 8 <= g1; g += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = q[(int64_t)(g + u) * stride];
#pragma unroll
          for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; g < g1; ++g) s += q[(int64_t)g * stride];
      } else {  // deviance and the other scalars: compensated, in the same order
        for (; g + 8 <= g1; g += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = q[(int64_t)(g + u) * stride];
#pragma unroll
          for (int u = 0; u < 8; ++u) neumaier_add(s, c, v[u]);
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
template <int FAM, int LNK>
__global__ void __launch_bounds__(256) stats_kernel(StatsArgs a) {
  __shared__ double red[4][NS];
  RowAcc acc;
#pragma unroll
  for (int k = 0; k < NS; ++k) acc.s[k] = 0.0;
  const int64_t per = (a.n + gridDim.x - 1) / gridDim.x;
  const int64_t lo = per * blockIdx.x, hi = (lo + per < a.n) ? lo + per : a.n;
  const double ybar = a.ybar_dev ? *a.ybar_dev : a.ybar;
  for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const double m = a.m ? a.m[i] : 1.0;
    const double pw = a.prior ? a.prior[i] : 1.0;
    double eta = 0.0;
    if (a.X) {  // LM residuals: X*coefs in predict_kernel's order (LM.scala:173-174)
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
// otherwise reruns the residual pass at its own).  Four waves; in every wave lane i is row i.
// The factorization runs right-looking: step k takes column k's pivot and scales the column, then
// subtracts L(i,k) L(j,k) from every trailing element (i, j) -- each element still receives its
// subtractions in ascending k, exactly chol_factor's left-looking order, but one step's subtractions
// are independent: waves 0-2 split the trailing columns (j mod 3), each forming the pivot and L(:,k)
// itself (the same operations, so the same values) and taking L(j,k) from its own lanes by readlane;
// wave 3 runs the forward sweep L t = b one column behind.  One barrier per step.  The back
// substitution is a column sweep on one wave (the host chol_solve's order).  The first forms -- one
// wave, left-looking, one LDS read and branch per subtraction -- took 37 us at p = 20; one wave
// right-looking 26 us (the chain of 20 pivots at single-wave latency plus all the updates).
// Out: beta[p]; aux[0] = sum y / rows (LM.scala:167-168), aux[1] = 1 where the host would leave
// Cholesky (a non-positive pivot, or the pivot ratio below LU_SWITCH_RATIO: solve.cpp chol_pivot_ratio).
__device__ __forceinline__ double lane_bcast(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l), __builtin_amdgcn_readlane(__double2loint(v), l));
}
__global__ void __launch_bounds__(256) lm_chol_kernel(const double* __restrict__ packed, int p, double ratio_min,
                                                      double* __restrict__ beta, double* __restrict__ aux) {
#pragma clang fp contract(off)
  constexpr int LD = 65, U = 8, NUPD = 3;  // A(r, c) at A[c LD + r]; waves 0..NUPD-1 update, wave NUPD solves
  __shared__ double A[64 * LD], dg[64], tsh[64];
  __shared__ int fail_sh;
  const int i = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool row = i < p;
  const int64_t tri = (int64_t)p * (p + 1) / 2;
  for (int e = threadIdx.x; e < p * p; e += 256) {  // unpack_gram: A(r, c) = packed[max(r, c) (max + 1) / 2 + min(r, c)]
    const int r = e % p, c = e / p, hi = r > c ? r : c, lo = r > c ? c : r;
    A[c * LD + r] = packed[hi * (hi + 1) / 2 + lo];
  }
  if (threadIdx.x < 64 && row) dg[i] = packed[(int64_t)i * (i + 1) / 2 + i];
  if (threadIdx.x == 0) fail_sh = 0;
  double ti = row ? packed[tri + i] : 0.0;  // wave NUPD: the forward sweep's t
  __syncthreads();
  for (int k = 0; k < p; ++k) {  // chol_factor
    const double d = A[k * LD + k];
    const double aik = A[k * LD + i];
    if (!(d > 0.0) || !isfinite(d)) {  // every wave sees the same d: a uniform exit
      if (threadIdx.x == 0) fail_sh = 1;
      break;
    }
    const double sq = sqrt(d);
    const double inv = 1.0 / sq;
    const double lik = (i == k) ? sq : aik * inv;  // L(i, k), lanes i >= k
    if (wv < NUPD) {
      // A(i, j) -= L(i, k) L(j, k) for this wave's trailing columns j = k+1+wv, k+1+wv+NUPD, ...; L(j, k) == 0 skipped
      for (int j0 = k + 1 + wv; j0 < p; j0 += NUPD * U) {
        double l[U], x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = j0 + NUPD * u < p ? j0 + NUPD * u : p - 1;
          l[u] = lane_bcast(lik, j);
          x[u] = A[j * LD + i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = j0 + NUPD * u;
          if (j < p) {  // wave-uniform
            const double nv = x[u] - lik * l[u];
            A[j * LD + i] = (i >= j && row && l[u] != 0.0) ? nv : x[u];
          }
        }
      }
    } else {
      // L t = b, column k: t_k /= L(k, k); t_i -= L(i, k) t_k, i > k
      const double tk = lane_bcast(ti / sq, k);
      if (i == k) ti = tk;
      if (i > k && row) ti -= lik * tk;
    }
    __syncthreads();
    // column k of L into A after every wave has read A(k, k) and A(:, k) (only the solves and the
    // pivot ratio read it again; the next step reads column k + 1)
    if (wv == 0 && i >= k && row) A[k * LD + i] = lik;
  }
  __syncthreads();
  const int fail = fail_sh;
  if (!fail) {
    if (wv == NUPD) tsh[i] = ti;
    __syncthreads();
    if (wv == 0) {
      double tb = tsh[i];
      for (int r = p - 1; r >= 0; --r) {  // L' x = t: x_r = t_r / L(r, r); t_i -= L(r, i) x_r, i < r
        const double xr = lane_bcast(tb / A[i * LD + i], r);
        if (i == r) tb = xr;
        if (i < r) tb -= A[i * LD + r] * xr;
      }
      if (row) beta[i] = tb;
    }
  }
  if (threadIdx.x == 0) {
    double r = 1.0;  // chol_pivot_ratio
    if (!fail)
      for (int j = 0; j < p; ++j) {
        const double l = A[j * LD + j], a = dg[j];
        if (a > 0.0) r = fmin(r, (l * l) / a);
      }
    aux[0] = packed[tri + p + S_DEV] / packed[tri + p + S_SUMW];
    aux[1] = (fail || r < ratio_min) ? 1.0 : 0.0;
  }
}

// The stats partials [nparts][NS] summed on the device into out[NS] (no D2H of the partials):
// thread (segment s, scalar k) sums partials [s n / 32, (s+1) n / 32) in order, Neumaier-compensated,
// then thread k adds the 32 segment sums and their compensations in segment order.
__global__ void __launch_bounds__(256) reduce_stats_kernel(const double* __restrict__ part, int nparts,
                                                           double* __restrict__ out) {
  __shared__ double ss[32][NS], cs[32][NS];
  const int k = threadIdx.x % NS, sg = threadIdx.x / NS;
  const int g0 = (int)((int64_t)nparts * sg / 32), g1 = (int)((int64_t)nparts * (sg + 1) / 32);
  double s = 0.0, c = 0.0;
  int g = g0;
  for (; g + 8 <= g1; g += 8) {  // 8 loads in flight ahead of the ordered compensated adds
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(g + u) * NS + k];
#pragma unroll
    for (int u = 0; u < 8; ++u) neumaier_add(s, c, v[u]);
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
  }
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
bool pass_uses_split(int P16, int fused_split, int64_t ld) {
  const int thr = fused_split == 1 ? ((P16 & 1) ? K1R_MIN_ODD : K1R_MIN_P16) : fused_split;
  return fused_split != 0 && P16 >= 5 && P16 >= thr && ld * 24 + 4096 < ((int64_t)1 << 32);
}
int pass_variant(int p, int fused_split, int64_t ld) {
  int P16 = (p + 15) / 16;
  if ((P16 & 1) && !pass_uses_split(P16, fused_split, ld)) ++P16;
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
    case 6: return wg_per_cu_t<6>();
    case 8: return wg_per_cu_t<8>();
    case 10: return wg_per_cu_t<10>();
    case 12: return wg_per_cu_t<12>();
    case 14: return wg_per_cu_t<14>();
    default: return wg_per_cu_t<16>();
  }
}

template <int P16>
static hipError_t launch_pass_p(const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  static_assert(P16 % 2 == 0, "K1: even column-block counts (odd ones: fused_odd.hip)");
  if constexpr (P16 >= 6)
    if (pass_uses_split(P16, a.fused_split, a.ld)) return launch_pass_r_fl<P16>(a, grid, st, e0, e1);
  const dim3 g(grid), b(64 * Geo<P16>::NW);
  const int mode_fam = (a.mode == MODE_LM_GRAM) ? FAM_GAUSSIAN : a.family;
  const int mode_lnk = (a.mode == MODE_LM_GRAM) ? LNK_IDENTITY : a.link;
  if (mode_fam == FAM_BINOMIAL && mode_lnk == LNK_LOGIT)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_BINOMIAL, LNK_LOGIT>), g, b, 0, st, e0, e1, 0, a);
  else if (mode_fam == FAM_BINOMIAL && mode_lnk == LNK_PROBIT)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_BINOMIAL, LNK_PROBIT>), g, b, 0, st, e0, e1, 0, a);
  else if (mode_fam == FAM_BINOMIAL)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_BINOMIAL, LNK_CLOGLOG>), g, b, 0, st, e0, e1, 0, a);
  else if (mode_fam == FAM_GAUSSIAN)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_GAUSSIAN, LNK_IDENTITY>), g, b, 0, st, e0, e1, 0, a);
  else if (mode_fam == FAM_POISSON)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_POISSON, LNK_LOG>), g, b, 0, st, e0, e1, 0, a);
  else if (mode_fam == FAM_GAMMA)
    hipExtLaunchKernelGGL((irls_pass_kernel<P16, FAM_GAMMA, LNK_INVERSE>), g, b, 0, st, e0, e1, 0, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_pass(int P16, const PassArgs& a, int grid, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
  if ((P16 & 1) && P16 >= 5) {
    // odd counts exist only as K1r: refuse a pass that may not run it (pass_variant rounds those up)
    if (!pass_uses_split(P16, a.fused_split, a.ld)) return hipErrorInvalidValue;
    return launch_pass_odd(P16, a, grid, st, e0, e1);
  }
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

hipError_t launch_lm_chol(const double* packed, int p, double ratio_min, double* beta, double* aux, hipStream_t st) {
  if (p < 1 || p > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(lm_chol_kernel, dim3(1), dim3(256), 0, st, packed, p, ratio_min, beta, aux);
  return hipGetLastError();
}

hipError_t launch_reduce_stats(const double* part, int nparts, double* out, hipStream_t st) {
  hipLaunchKernelGGL(reduce_stats_kernel, dim3(1), dim3(32 * NS), 0, st, part, nparts, out);
  return hipGetLastError();
}

hipError_t launch_stats(const StatsArgs& a, int grid, hipStream_t st) {
  const dim3 gr(grid), bl(256);
  if (a.mode == MODE_LM_RESID || (a.family == FAM_GAUSSIAN && a.link == LNK_IDENTITY))
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
                         hipEvent_t e1) {
  const int64_t total = (int64_t)p * (p + 1) / 2 + p + NS;
  int blocks = (int)((total + RED_EL - 1) / RED_EL);
  if (blocks > 8192) blocks = 8192;
  hipExtLaunchKernelGGL(reduce_partials_kernel, dim3(blocks), dim3(256), 0, st, nullptr, e1, 0, part, stride, nparts, p, P16,
                        out);
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
