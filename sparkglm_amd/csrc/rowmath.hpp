// rowmath.hpp -- per-row family/link arithmetic of the IRLS pass (device side).
//
// Mirrors the reference's elementwise stage operation-for-operation:
//   link / lPrime / unlink  GLM.scala:190-251   (logit, probit, cloglog)
//   varianceBinomial        GLM.scala:125-129
//   w = 1/(V g'^2), z = eta + (y - mu) g' - offset      GLM.scala:289-290, 370-371
//   devBinomial row value   GLM.scala:166-167   (summed, times 2 on the host)
//   pearsonCalc             GLM.scala:90-101
//   llBinomial              GLM.scala:132-143   (Breeze Binomial(m.toInt, mu).logProbabilityOf)
// Extension families (gaussian/identity, poisson/log, gamma/inverse, prior weights)
// follow R's family objects on the same skeleton.
#pragma once
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace sglm {

// Breeze Gaussian(0,1) as used by the probit link.
__device__ __forceinline__ double norm_cdf(double x) { return 0.5 * (1.0 + erf(x / sqrt(2.0))); }
__device__ __forceinline__ double norm_icdf(double q) { return 0.0 + 1.0 * sqrt(2.0) * erfinv(2.0 * q - 1.0); }
__device__ __forceinline__ double norm_pdf(double x) {
  double d = (x - 0.0) / 1.0;
  return exp(-d * d / 2.0 - (log(sqrt(2.0 * M_PI)) + log(1.0)));
}

// A polynomial coefficient materialised in an SGPR pair at its point of use (two s_mov_b32 on
// the scalar unit): without this the compiler hoists every coefficient of the fast paths out
// of the pass kernels' main loops into VGPRs, where they crowd out the Gram accumulators and
// spill to scratch -- and a scratch reload's vmcnt wait drains the LDS-DMA pipeline.
__device__ __forceinline__ double sc(double c) {
  asm volatile("" : "+s"(c));
  return c;
}

// Reciprocal of a positive normal x: v_rcp_f64 plus two Newton steps (quadratic convergence
// from the hardware estimate), ~1 ulp -- the fast paths below use it in place of the IEEE
// division sequence (div_scale / div_fmas / div_fixup), which they never need: their operands
// are bounded away from 0, denormals and infinity by the fast-path range checks.
__device__ __forceinline__ double rcp_pos(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(fma(-x, r, 1.0), r, r);
  return fma(fma(-x, r, 1.0), r, r);
}

// Natural log of a positive finite x (normal or denormal), ~2 ulp: x = m 2^k with
// m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m - 1)/(m + 1), |s| <= 0.1716, as
// 2s (1 + s^2/3 + ... + s^18/19) (truncation < 3e-17 relative).  The row fast paths use it
// for the deviance terms instead of libm's double-double log / log1p (about 3x fewer
// instructions); the per-row values differ from libm's by a few ulp, far inside the 1e-9
// parity tolerance on the summed deviance.
__device__ __forceinline__ double log_pos(double x) {
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
  int k = __builtin_amdgcn_frexp_exp(x);
  if (m < sc(0.70710678118654752440)) {
    m = m + m;
    k -= 1;
  }
  const double f = m - 1.0;
  const double s = f * rcp_pos(m + 1.0);
  const double z = s * s;
  // (Horner: Estrin's scheme, dependency depth 4 instead of 9, measured +-0 -- not kept)
  double q = sc(1.0 / 19.0);
  q = fma(q, z, sc(1.0 / 17.0));
  q = fma(q, z, sc(1.0 / 15.0));
  q = fma(q, z, sc(1.0 / 13.0));
  q = fma(q, z, sc(1.0 / 11.0));
  q = fma(q, z, sc(1.0 / 9.0));
  q = fma(q, z, sc(1.0 / 7.0));
  q = fma(q, z, sc(1.0 / 5.0));
  q = fma(q, z, sc(1.0 / 3.0));
  const double lm = fma(2.0 * s, z * q, 2.0 * s);
  const double kd = (double)k;
  return fma(kd, sc(6.93147180559945286227e-01), fma(kd, sc(2.31904681384629955842e-17), lm));
}

// exp(x) for |x| < 708 (the fast paths' range checks guarantee it), ~2 ulp: x = k ln2 + r,
// |r| <= ln2/2, Taylor series to r^13 (truncation < 5e-18 relative), scaled by 2^k.  No
// overflow / underflow / NaN handling -- libm's exp carries that on every call.
__device__ __forceinline__ double exp_small(double x) {
  const double kf = rint(x * sc(1.44269504088896338700));
  double r = fma(-kf, sc(6.93147180559945286227e-01), x);
  r = fma(-kf, sc(2.31904681384629955842e-17), r);
  double q = sc(1.0 / 6227020800.0);  // 1/13!
  q = fma(q, r, sc(1.0 / 479001600.0));
  q = fma(q, r, sc(1.0 / 39916800.0));
  q = fma(q, r, sc(1.0 / 3628800.0));
  q = fma(q, r, sc(1.0 / 362880.0));
  q = fma(q, r, sc(1.0 / 40320.0));
  q = fma(q, r, sc(1.0 / 5040.0));
  q = fma(q, r, sc(1.0 / 720.0));
  q = fma(q, r, sc(1.0 / 120.0));
  q = fma(q, r, sc(1.0 / 24.0));
  q = fma(q, r, sc(1.0 / 6.0));
  q = fma(q, r, 0.5);
  q = fma(q, r, 1.0);
  q = fma(q, r, 1.0);
  return __builtin_amdgcn_ldexp(q, (int)kf);
}

__device__ __forceinline__ double link_fn(int fam, int lnk, double mu, double m) {
  if (fam == FAM_BINOMIAL) {
    if (lnk == LNK_LOGIT) return log(mu / (m + (-1.0 * mu)));
    if (lnk == LNK_PROBIT) return norm_icdf(mu / m);
    return log(-1.0 * log(1.0 + (-1.0 * (mu / m))));
  }
  if (fam == FAM_GAUSSIAN) return mu;
  if (fam == FAM_POISSON) return log(mu);
  return 1.0 / mu;
}

__device__ __forceinline__ double unlink_fn(int fam, int lnk, double eta, double m) {
  if (fam == FAM_BINOMIAL) {
    if (lnk == LNK_LOGIT) return m / (1.0 + exp(-1.0 * eta));
    if (lnk == LNK_PROBIT) return m * norm_cdf(eta);
    return m * (1.0 + (-1.0 * exp(-exp(eta))));
  }
  if (fam == FAM_GAUSSIAN) return eta;
  if (fam == FAM_POISSON) return exp(eta);
  return 1.0 / eta;
}

__device__ __forceinline__ double lprime_fn(int fam, int lnk, double mu, double m) {
  if (fam == FAM_BINOMIAL) {
    if (lnk == LNK_LOGIT) return m / (mu * (m + (-1.0 * mu)));
    if (lnk == LNK_PROBIT) return 1.0 / (m * norm_pdf(norm_icdf(mu / m)));
    return 1.0 / ((mu + (-1.0 * m)) * log(1.0 + (-1.0 * (mu / m))));
  }
  if (fam == FAM_GAUSSIAN) return 1.0;
  if (fam == FAM_POISSON) return 1.0 / mu;
  return -1.0 / (mu * mu);
}

__device__ __forceinline__ double variance_fn(int fam, double mu, double m) {
  if (fam == FAM_BINOMIAL) return mu * (1.0 + (-1.0 * (mu / m)));
  if (fam == FAM_GAUSSIAN) return 1.0;
  if (fam == FAM_POISSON) return mu;
  return mu * mu;
}

// Breeze Binomial(n, p).logProbabilityOf(k) with n = m.toInt, k = y.toInt, p = mu.
__device__ __forceinline__ double binom_logpmf(double mval, double mu, double yval, double& bad) {
  int n = (int)mval, k = (int)yval;
  if (n <= 0 || k < 0 || k > n || mu < 0.0) { bad += 1.0; return 0.0; }
  if (mu == 0.0) return k == 0 ? 0.0 : -INFINITY;
  if (mu == 1.0) return k == n ? 0.0 : -INFINITY;
  return lgamma(n + 1.0) - lgamma(k + 1.0) - lgamma(n - k + 1.0) + k * log(mu) + (n - k) * log1p(-mu);
}

// Compensated (Neumaier) accumulation for the last, widest levels of the scalar reductions: at
// 1e9 rows a plain sum of ~256-2048 partials of a ~1e9 deviance carries ~1e-6 of rounding --
// GLM.scala:281's absolute tol -- so the iteration count would follow the summation order.
__device__ __forceinline__ void neumaier_add(double& s, double& c, double x) {
  const double t = s + x;
  c += (fabs(s) >= fabs(x)) ? (s - t) + x : (x - t) + s;
  s = t;
}

struct RowAcc {
  double s[NS];
};

// Poisson counts y < POIS_TAB that are integers take their per-row functions of y from tables
// built once per workgroup in LDS with the reference's own expressions (poisson_init_table,
// poisson_ylogy_table below).
constexpr int POIS_TAB = 256;

// Unit deviance row value: devBinomial (GLM.scala:166-167) and the R families; the
// family factor (2 for binomial / poisson / gamma) is applied on the host after summing.
__device__ __forceinline__ double unit_dev(int fam, double y, double mu, double m, double pw) {
  if (fam == FAM_BINOMIAL) {
    double my = m + (-1.0 * y);
    return pw * ((y * log(fmax(y, 1.0) / mu)) + (my * log(fmax(my, 1.0) / (m + (-1.0 * mu)))));
  }
  if (fam == FAM_GAUSSIAN) {
    double e = y - mu;
    return pw * (e * e);
  }
  if (fam == FAM_POISSON) return pw * ((y > 0.0 ? y * log(y / mu) : 0.0) - (y - mu));
  return pw * (-(log(y / mu) - (y - mu) / mu));
}

// The reference operation order (zwCreateBinomial GLM.scala:359-395, devBinomial :162-170)
// for every row the fast paths below do not take: init modes, m != 1, probit / cloglog, and
// rows outside the fast paths' ranges.  Out of line: its libm calls' constants would otherwise
// be hoisted into the pass kernels' main loops and take registers from the Gram accumulators.
struct RowWZ {
  double w, wz, dev;
};
__device__ __noinline__ RowWZ pass_row_ref(int fam, int lnk, int mode, double eta, double y, double m, double off,
                                           double pw, double mu0) {
  double mu;
  if (mode == MODE_IRLS) {
    mu = unlink_fn(fam, lnk, eta, m);
  } else {
    eta = link_fn(fam, lnk, mu0, m);  // offset ignored at init (GLM.scala:264-270)
    mu = (mode == MODE_INIT_SINGLE) ? mu0 : unlink_fn(fam, lnk, eta, m);
  }
  const double g = lprime_fn(fam, lnk, mu, m);
  const double v = variance_fn(fam, mu, m);
  RowWZ r;
  r.w = pw * (1.0 / (v * (g * g)));
  const double z = (eta + ((y + (-1.0 * mu)) * g)) + (-1.0 * off);
  r.wz = r.w * z;
  // fitMultipleBinomial re-derives mu = unlink(link(ybar)) only inside zwCreateBinomial; its
  // null deviance is taken at mu0 = ybar itself (GLM.scala:424-444)
  r.dev = unit_dev(fam, y, mode == MODE_IRLS ? mu : mu0, m, pw);
  return r;
}

// The initial pass of a binomial fit without m (GLM.scala:263-272, 429-444): mu = mu0
// (fitSingle) or unlink(link(mu0)) (fitMultiple) is the same for every row, so link, lPrime and
// the variance are invariants of the pass; per row only z and the deviance remain.
// max(y, 1) = max(1 - y, 1) = 1 for 0 <= y <= 1, so devBinomial's logs are invariant too -- the
// expressions are the reference's own, operation for operation (pass_row_ref), so the rows come
// out bitwise pass_row_ref's.  v = {e0, mu, g, w0, l1, l0}.
struct InitConst {
  double v[6];
};
__device__ __forceinline__ InitConst init_const(int fam, int lnk, int mode, double mu0) {
  InitConst c;
  const double e0 = link_fn(fam, lnk, mu0, 1.0);
  const double mu = (mode == MODE_INIT_SINGLE) ? mu0 : unlink_fn(fam, lnk, e0, 1.0);
  const double g = lprime_fn(fam, lnk, mu, 1.0);
  c.v[0] = e0;
  c.v[1] = mu;
  c.v[2] = g;
  c.v[3] = 1.0 / (variance_fn(fam, mu, 1.0) * (g * g));
  c.v[4] = fam == FAM_BINOMIAL ? log(1.0 / mu0) : 0.0;
  c.v[5] = fam == FAM_BINOMIAL ? log(1.0 / (1.0 + (-1.0 * mu0))) : 0.0;
  return c;
}
// the fused kernels' initial passes take these constants from LDS (computed once per workgroup)
__device__ __forceinline__ bool init_fast_row(int fam, int mode, bool has_m) {
  return fam == FAM_BINOMIAL && (mode == MODE_INIT_SINGLE || mode == MODE_INIT_MULTI) && !has_m;
}
__device__ __forceinline__ void pass_row_init(const double* c, double y, double off, double pw, double& w, double& wz,
                                              double& s_dev, double& s_aux) {
  w = pw * c[3];
  const double z = (c[0] + ((y + (-1.0 * c[1])) * c[2])) + (-1.0 * off);
  wz = w * z;
  const double my = 1.0 + (-1.0 * y);
  s_dev += pw * ((y * c[4]) + (my * c[5]));
  s_aux += pw;
}

// The row stage of the fused pass (zwCreateBinomial, GLM.scala:359-395 / the single-
// partition loop body GLM.scala:282-301): w and w*z for the Gramian, and the deviance.
// LM gram mode: w = 1, z = y, and the sums of y and of rows (LM.scala:142-155, 167).
// small_exp and init_fast are compile-time constants at every call site.
// small_exp selects exp_small over libm's exp.  Every narrow variant (p <= 64) passes true: round 4
// measured it -1 % at p <= 32 and +4 % at p = 64 on that round's narrow kernel; round 5's rework of
// the narrow pass (row stage at raised issue priority, block pairs at p > 32) set it for every width
// without a separate p = 64 A/B of this choice.  The fused / wide kernels leave it off (neutral).
// ylogy (the narrow kernel's Poisson IRLS passes): an LDS table of k log k for the integer counts
// k < POIS_TAB (poisson_ylogy_table), so that those rows need no log: the Poisson unit deviance
// y log(y / mu) - (y - mu) = (y log y - y eta) - (y - mu) with y log y looked up.  The deviance stays
// a per-row sum of terms of the size of the row's own deviance -- what GLM.scala:452's absolute tol
// on the change needs (a round-3 form summed -y eta - (y - mu) per row and added sum y log y once
// per pass: with counts ~1e3 over 1e8 rows its terms reached ~1e12 in total and their rounding,
// ~1e-4, swamped tol 1e-6).  Other rows (non-integer or large y) take log_pos.
__device__ __forceinline__ void pass_row(int fam, int lnk, int mode, double eta, double y, double m, double off,
                                         double pw, double mu0, double ybar, bool has_m, double& w, double& wz,
                                         double& s_dev, double& s_aux, bool small_exp = false,
                                         bool init_fast = false, const double* ylogy = nullptr) {
  (void)ybar;
  if (fam == FAM_BINOMIAL && lnk == LNK_LOGIT && mode == MODE_IRLS && !has_m && fabs(eta) < 8.0 && y >= 0.0 &&
      y <= 1.0) {
    // Logit, m = 1: the reference's expressions (GLM.scala:190-204, 125-129, 162-170, 289-290)
    // in an algebraically identical form with one exp, one division and one log1p:
    //   t = 1/(1+e), e = exp(-eta):  mu = t,  V = e t^2,  g' = 1/V,  w = V,  w*z = V (eta - off) + (y - mu)
    //   dev row = y log(1/mu) + (1-y) log(1/(1-mu)) = log1p(e) + (1-y) eta
    // Inside |eta| < 8 both forms agree to ~1e-13 relative per row (1 - mu >= 3e-4, no
    // cancellation); outside it, and for m != 1, the reference operation order below applies.
    // u = 1 + e lies in (1, 2982): t = 1/u by rcp_pos, and log1p(e) = log(u) + (e - (u - 1))/u
    // (the rounding of u corrected to first order, as libm's log1p does).
    const double e = small_exp ? exp_small(-eta) : exp(-eta);
    const double u = 1.0 + e;
    const double t = rcp_pos(u);
    const double v = e * t * t;
    w = pw * v;
    wz = pw * (v * (eta - off) + (y - t));
    s_dev += pw * (fma(e - (u - 1.0), t, log_pos(u)) + (1.0 - y) * eta);
    s_aux += pw;
    return;
  }
  if (fam == FAM_POISSON && mode == MODE_IRLS && fabs(eta) < 700.0 && y >= 0.0 && y < 1e300) {
    // Poisson / log (R's poisson()): mu = exp(eta), g' = 1/mu, V = mu, so
    //   w = 1/(V g'^2) = mu,  w*z = mu (eta - off) + (y - mu),
    //   dev row = y log(y/mu) - (y - mu) with log(y/mu) = log(y) - eta
    // -- one exp and one log (or a table look-up), no divisions; the reference operation order
    // (below) agrees to a few ulp per row, and it still runs where exp could overflow.
    const double mu = small_exp ? exp_small(eta) : exp(eta);
    w = pw * mu;
    wz = pw * (mu * (eta - off) + (y - mu));
    double d0;
    if (ylogy && y < (double)POIS_TAB && y == floor(y)) d0 = ylogy[(int)y] - y * eta;
    else d0 = y > 0.0 ? y * (log_pos(y) - eta) : 0.0;
    s_dev += pw * (d0 - (y - mu));
    s_aux += pw;
    return;
  }
  if (fam == FAM_GAMMA && mode == MODE_IRLS && eta > 1e-150 && eta < 1e150 && y > 1e-150 && y < 1e150) {
    // Gamma / inverse (R's Gamma()): mu = 1/eta, g' = -1/mu^2, V = mu^2, so
    //   w = mu^2,  w*z = mu^2 (eta - off) - (y - mu),
    //   dev row = -(log(y/mu) - (y - mu)/mu) = -(log(y eta) - (y eta - 1))
    // -- one reciprocal and one log instead of four divisions and a log (the range checks keep
    // eta, y and y eta normal and finite for rcp_pos / log_pos).
    const double mu = rcp_pos(eta);
    const double mu2 = mu * mu;
    const double ye = y * eta;
    w = pw * mu2;
    wz = pw * (mu2 * (eta - off) - (y - mu));
    s_dev += pw * (-(log_pos(ye) - (ye - 1.0)));
    s_aux += pw;
    return;
  }
  if (mode == MODE_LM_GRAM) {
    w = 1.0;
    wz = y;
    s_dev += y;
    s_aux += 1.0;
    return;
  }
  if (init_fast && fam == FAM_BINOMIAL && mode != MODE_IRLS && mode != MODE_LM_GRAM && !has_m && y >= 0.0 &&
      y <= 1.0) {
    // (init_fast: set by the narrow kernel's non-IRLS instantiation only, whose loop the
    // invariants are hoisted out of; the fused kernels take them from LDS, init_const below.)
    const InitConst c = init_const(fam, lnk, mode, mu0);
    pass_row_init(c.v, y, off, pw, w, wz, s_dev, s_aux);
    return;
  }
  const RowWZ r = pass_row_ref(fam, lnk, mode, eta, y, m, off, pw, mu0);
  w = r.w;
  wz = r.wz;
  s_dev += r.dev;
  s_aux += pw;
}

// Logit with m = 1, in-pass final statistics (PassArgs::stats_in_pass): the IRLS row stage of
// pass_row plus stats_row's pearsonCalc / llBinomial terms at the same mu, sharing one exp, one
// reciprocal and one log -- the pass then needs no eta store and no stats_kernel pass.  Rows
// outside the fast range take both reference-order functions.
__device__ __forceinline__ void pass_row_logit_stats(double eta, double y, double off, double pw, double& w, double& wz,
                                                     double& s_dev, double& s_aux, double& s_pear, double& s_ll,
                                                     double& s_bad, bool small_exp);

// The reference operation order of the final statistics (pearsonCalc GLM.scala:90-101,
// llBinomial :132-143, devBinomial :162-170, the R families' loglik ingredients), out of line
// like pass_row_ref: rows the inline fast path of stats_row does not take.
__device__ __noinline__ RowAcc stats_row_ref(int fam, int lnk, int mode, double eta, double y, double m, double pw,
                                             double mu0, bool has_m) {
  RowAcc acc;
#pragma unroll
  for (int k = 0; k < NS; ++k) acc.s[k] = 0.0;
  // init modes (a fit that stops before its first solve): the statistics at mu0 itself, as
  // pearsonCalc / llBinomial see the broadcast ybar (GLM.scala:424-426, 465-466)
  const double mu = (mode == MODE_IRLS) ? unlink_fn(fam, lnk, eta, m) : mu0;
  const double v = variance_fn(fam, mu, m);
  const double r = y + (-1.0 * mu);
  acc.s[S_DEV] += unit_dev(fam, y, mu, m, pw);
  acc.s[S_PEARSON] += pw * (r * r) / v;
  acc.s[S_SUMW] += pw;
  if (fam == FAM_BINOMIAL) {
    double bad = 0.0, ll;
    if (has_m) {
      ll = binom_logpmf(m, mu, y, bad);
    } else {  // m == 1: the lgamma terms vanish; same special cases as Breeze
      const int k = (int)y;
      if (k < 0 || k > 1 || mu < 0.0) { bad = 1.0; ll = 0.0; }
      else if (mu == 0.0) ll = k == 0 ? 0.0 : -INFINITY;
      else if (mu == 1.0) ll = k == 1 ? 0.0 : -INFINITY;
      else ll = k * log(mu) + (1 - k) * log1p(-mu);
    }
    acc.s[S_LL] += pw * ll;
    acc.s[S_BAD] += bad;
  } else if (fam == FAM_GAUSSIAN) {
    acc.s[S_LL] += log(pw);
  } else if (fam == FAM_POISSON) {
    acc.s[S_LL] += pw * (y * log(mu) - mu - lgamma(y + 1.0));
  } else {
    acc.s[S_LL] += pw * log(y);
    acc.s[S_AUX0] += pw * (y / mu);
    acc.s[S_AUX1] += pw * log(mu);
  }
  return acc;
}

// Final statistics of one row at the converged mu: pearsonCalc (GLM.scala:90-101),
// llBinomial (GLM.scala:132-143) and the extension families' loglik ingredients; LM
// mode: SSE / SSR / SST terms of rowPartitionedSSE (LM.scala:172-175) with eta = X*coefs.
__device__ __forceinline__ void stats_row(int fam, int lnk, int mode, double eta, double y, double m, double pw,
                                          double mu0, double ybar, bool has_m, RowAcc& acc) {
  if (mode == MODE_LM_RESID) {
    const double e = y - eta, t = eta + (-1.0 * ybar), b = y + (-1.0 * ybar);
    acc.s[S_DEV] += e * e;
    acc.s[S_PEARSON] += t * t;
    acc.s[S_LL] += b * b;
    acc.s[S_SUMW] += 1.0;
    return;
  }
  if (fam == FAM_BINOMIAL && lnk == LNK_LOGIT && mode == MODE_IRLS && !has_m && fabs(eta) < 8.0 && y >= 0.0 &&
      y <= 1.0) {
    // Logit, m = 1, the pass's fast-path forms (pass_row): mu = t = 1/(1+e), e = exp(-eta),
    // V = mu(1 - mu) = e t^2, unit deviance log1p(e) + (1-y) eta, and Breeze's
    // Binomial(1, mu).logProbabilityOf(k) = k log mu + (1-k) log(1-mu) with log mu = -log1p(e),
    // log(1-mu) = -eta - log1p(e); |eta| < 8 keeps mu off 0 and 1 (no special cases, k in {0, 1}).
    const double e = exp_small(-eta);
    const double u = 1.0 + e;
    const double t = rcp_pos(u);
    const double L = fma(e - (u - 1.0), t, log_pos(u));
    const double v = e * t * t;
    const double r = y - t;
    acc.s[S_DEV] += pw * (L + (1.0 - y) * eta);
    acc.s[S_PEARSON] += pw * (r * r) * rcp_pos(v);
    acc.s[S_SUMW] += pw;
    acc.s[S_LL] += pw * ((int)y == 1 ? -L : -L - eta);
    return;
  }
  const RowAcc r = stats_row_ref(fam, lnk, mode, eta, y, m, pw, mu0, has_m);
#pragma unroll
  for (int k = 0; k < NS; ++k) acc.s[k] += r.s[k];
}

// Rows outside the in-pass statistics' fast ranges: both reference-order functions and the
// family's statistics slots (s2, s3, s4: StatsSlots), in ONE out-of-line call -- two calls (or
// an inlined lgamma) around the kernel's live Gram accumulators made the compiler spill them.
struct RowStats {
  double w, wz, dev, s2, s3, s4;
};
__device__ __noinline__ RowStats stats_row_fallback(int fam, int lnk, double eta, double y, double off, double pw) {
  const RowWZ r = pass_row_ref(fam, lnk, MODE_IRLS, eta, y, 1.0, off, pw, 0.0);
  const RowAcc a = stats_row_ref(fam, lnk, MODE_IRLS, eta, y, 1.0, pw, 0.0, false);
  RowStats o;
  o.w = r.w;
  o.wz = r.wz;
  o.dev = r.dev;
  o.s2 = a.s[S_PEARSON];
  if (fam == FAM_BINOMIAL) {
    o.s3 = a.s[S_LL];
    o.s4 = a.s[S_BAD];
  } else if (fam == FAM_POISSON) {
    o.s3 = a.s[S_LL] + pw * lgamma(y + 1.0);  // the constant part is subtracted once per fit
    o.s4 = 0.0;
  } else {
    o.s3 = a.s[S_AUX0];
    o.s4 = a.s[S_LL] - a.s[S_AUX1];  // pw log y - pw log mu = pw log(y / mu)
  }
  return o;
}

__device__ __forceinline__ void pass_row_logit_stats(double eta, double y, double off, double pw, double& w, double& wz,
                                                     double& s_dev, double& s_aux, double& s_pear, double& s_ll,
                                                     double& s_bad, bool small_exp) {
  if (fabs(eta) < 8.0 && y >= 0.0 && y <= 1.0) {
    const double e = small_exp ? exp_small(-eta) : exp(-eta);
    const double u = 1.0 + e;
    const double t = rcp_pos(u);
    const double v = e * t * t;
    const double L = fma(e - (u - 1.0), t, log_pos(u));  // log1p(e) = -log(mu)
    w = pw * v;
    wz = pw * (v * (eta - off) + (y - t));
    s_dev += pw * (L + (1.0 - y) * eta);
    s_aux += pw;
    const double r = y - t;
    s_pear += pw * (r * r) * rcp_pos(v);
    s_ll += pw * ((int)y == 1 ? -L : -L - eta);
    return;
  }
  const RowStats r = stats_row_fallback(FAM_BINOMIAL, LNK_LOGIT, eta, y, off, pw);
  w = r.w;
  wz = r.wz;
  s_dev += r.dev;
  s_aux += pw;
  s_pear += r.s2;
  s_ll += r.s3;
  s_bad += r.s4;
}

// Poisson / log, in-pass final statistics: pass_row's fast path plus pearsonCalc (R's variance
// V = mu) and the mu-dependent part of R's dpois log-density, y log mu - mu with
// log mu = eta.  The per-row constant -lgamma(y + 1) does not depend on the fit: the initial pass
// sums pw lgamma(y + 1) once into S_AUX2 (init_stats_const) and the engine subtracts it.
// Slots: s2 = Pearson, s3 = loglik part, s4 unused.
__device__ __forceinline__ void pass_row_poisson_stats(double eta, double y, double off, double pw, double& w,
                                                       double& wz, double& s_dev, double& s_aux, double& s2,
                                                       double& s3, bool small_exp, const double* ylogy) {
  if (fabs(eta) < 700.0 && y >= 0.0 && y < 1e300) {
    const double mu = small_exp ? exp_small(eta) : exp(eta);
    w = pw * mu;
    wz = pw * (mu * (eta - off) + (y - mu));
    double d0;  // pass_row's Poisson unit deviance
    if (ylogy && y < (double)POIS_TAB && y == floor(y)) d0 = ylogy[(int)y] - y * eta;
    else d0 = y > 0.0 ? y * (log_pos(y) - eta) : 0.0;
    s_dev += pw * (d0 - (y - mu));
    s_aux += pw;
    const double r = y - mu;
    s2 += pw * (r * r) * rcp_pos(mu);
    s3 += pw * (y * eta - mu);
    return;
  }
  const RowStats r = stats_row_fallback(FAM_POISSON, LNK_LOG, eta, y, off, pw);
  w = r.w;
  wz = r.wz;
  s_dev += r.dev;
  s_aux += pw;
  s2 += r.s2;
  s3 += r.s3;
}

// Gamma / inverse, in-pass final statistics: pass_row's fast path plus pearsonCalc (V = mu^2:
// (y - mu)^2 / mu^2 = (y - mu)^2 eta^2) and R's Gamma loglik ingredients sum pw y / mu = sum pw y eta
// (S_AUX0) and sum pw log mu = sum pw log y - sum pw log(y eta) (S_AUX1: the pass sums the second
// term, which its deviance already evaluates; the fit-constant sum pw log y -- also S_LL itself --
// comes from the initial pass, init_stats_const).  Slots: s2 = Pearson, s3 = AUX0, s4 = log(y eta).
__device__ __forceinline__ void pass_row_gamma_stats(double eta, double y, double off, double pw, double& w,
                                                     double& wz, double& s_dev, double& s_aux, double& s2, double& s3,
                                                     double& s4) {
  if (eta > 1e-150 && eta < 1e150 && y > 1e-150 && y < 1e150) {
    const double mu = rcp_pos(eta);
    const double mu2 = mu * mu;
    const double ye = y * eta;
    const double L = log_pos(ye);
    w = pw * mu2;
    wz = pw * (mu2 * (eta - off) - (y - mu));
    s_dev += pw * (-(L - (ye - 1.0)));
    s_aux += pw;
    const double r = y - mu;
    s2 += pw * (r * r) * (eta * eta);
    s3 += pw * ye;
    s4 += pw * L;
    return;
  }
  const RowStats r = stats_row_fallback(FAM_GAMMA, LNK_INVERSE, eta, y, off, pw);
  w = r.w;
  wz = r.wz;
  s_dev += r.dev;
  s_aux += pw;
  s2 += r.s2;
  s3 += r.s3;
  s4 += r.s4;
}

// The per-fit constants of the in-pass statistics, summed by the initial pass into S_AUX2:
// Poisson sum pw lgamma(y + 1) (R's dpois), Gamma sum pw log y (R's dgamma).
__device__ __noinline__ double init_stats_const_ref(int fam, double y, double pw) {
  return fam == FAM_POISSON ? pw * lgamma(y + 1.0) : pw * log(y);
}
template <int FAM>
__device__ __forceinline__ double init_stats_const(double y, double pw) {
  if constexpr (FAM == FAM_POISSON || FAM == FAM_GAMMA) return init_stats_const_ref(FAM, y, pw);
  return 0.0;
}

// The initial pass of a Poisson fit (mu = mu0 for every row, GLM.scala:263-272, 429-444, R's
// poisson()): per row, pass_row_ref needs log(y / mu0) for the unit deviance, and the in-pass
// statistics' constant needs lgamma(y + 1) (init_stats_const) -- two libm calls on the 16 of 64
// lanes of a p = 64 narrow pass.  Counts y are small integers, so the two functions of k = y are
// tabulated once per workgroup for k < POIS_TAB with the very same expressions
// (tab[k] = (k > 0 ? k log(k / mu0) : 0) - (k - mu0), tab[T + k] = lgamma(k + 1)); a row then
// multiplies by its prior weight exactly where the reference expressions do, so the rows are
// bitwise pass_row_ref's.  Other rows (non-integer or large y) take the reference path.
__device__ __forceinline__ void poisson_init_table(double* tab, double mu0, int k) {
  const double y = (double)k;
  tab[k] = (y > 0.0 ? y * log(y / mu0) : 0.0) - (y - mu0);
  tab[POIS_TAB + k] = lgamma(y + 1.0);
}
// The IRLS passes' table (pass_row ylogy): k log k, 0 at k = 0.
__device__ __forceinline__ void poisson_ylogy_table(double* tab, int k) {
  const double y = (double)k;
  tab[k] = y > 0.0 ? y * log(y) : 0.0;
}
// w, w*z from the init constants c (init_const), the deviance and the statistics constant from
// the table; false: the row is not a tabulated count (caller takes the reference path)
__device__ __forceinline__ bool poisson_init_row(const double* c, const double* tab, double y, double off, double pw,
                                                 double& w, double& wz, double& s_dev, double& s_aux, double& s_lg) {
  if (!(y >= 0.0 && y < (double)POIS_TAB && y == floor(y))) return false;
  const int k = (int)y;
  w = pw * c[3];
  const double z = (c[0] + ((y + (-1.0 * c[1])) * c[2])) + (-1.0 * off);
  wz = w * z;
  s_dev += pw * tab[k];
  s_aux += pw;
  s_lg += pw * tab[POIS_TAB + k];
  return true;
}

// Dispatch of the in-pass statistics rows: three family-specific accumulators (s2, s3, s4) that
// the kernel stores into the slots stats_slots() names.
template <int FAM>
__device__ __forceinline__ void pass_row_stats(double eta, double y, double off, double pw, double& w, double& wz,
                                               double& s_dev, double& s_aux, double& s2, double& s3, double& s4,
                                               bool small_exp, const double* ylogy = nullptr) {
  if constexpr (FAM == FAM_BINOMIAL)
    pass_row_logit_stats(eta, y, off, pw, w, wz, s_dev, s_aux, s2, s3, s4, small_exp);
  else if constexpr (FAM == FAM_POISSON)
    pass_row_poisson_stats(eta, y, off, pw, w, wz, s_dev, s_aux, s2, s3, small_exp, ylogy);
  else
    pass_row_gamma_stats(eta, y, off, pw, w, wz, s_dev, s_aux, s2, s3, s4);
}
// slots of (s2, s3, s4): logit (Pearson, loglik, bad), Poisson (Pearson, loglik part, -),
// Gamma (Pearson, AUX0, sum pw log(y eta) -> AUX1 on the host)
template <int FAM>
struct StatsSlots {
  static constexpr int S2 = S_PEARSON;
  static constexpr int S3 = FAM == FAM_GAMMA ? S_AUX0 : S_LL;
  static constexpr int S4 = FAM == FAM_GAMMA ? S_AUX1 : (FAM == FAM_BINOMIAL ? S_BAD : -1);
};

}  // namespace sglm
