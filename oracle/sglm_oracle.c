/*
 * sglm_oracle.c -- CPU restatement of cafreeman/sparkGLM's lm()/glm() fitting path.
 *
 * TEST INFRASTRUCTURE ONLY (see sglm_oracle.h).  This file is the parity checker and
 * the timed CPU baseline ("port" of the reference algorithm, not the JVM).  It never
 * ships in the product path.
 *
 * Each function cites the reference line(s) it restates; paths are relative to the
 * reference root (src/main/scala/com/Alteryx/sparkGLM/...).  Arithmetic is written in
 * the same operation order as the Scala/Breeze expressions, with -ffp-contract=off, so
 * that the per-row values match a JVM evaluation up to libm ulps.
 *
 * Third-party arithmetic the reference reaches (not vendored, restated from its
 * published definition -- "as recalled", unverifiable offline):
 *   - Breeze 0.11.2 Gaussian(0,1): cdf(x) = .5*(1+erf(x/sqrt(2))),
 *     inverseCdf(q) = sqrt(2)*erfinv(2q-1), pdf(x) = exp(-x*x/2 - log(sqrt(2*Pi))).
 *   - Breeze Binomial(n,p).logProbabilityOf(k) =
 *     lgamma(n+1)-lgamma(k+1)-lgamma(n-k+1) + k*log(p) + (n-k)*log1p(-p), with the
 *     p==0 / p==1 special cases and require(n>=k), require(k>=0).
 *   - Breeze inv(): LAPACK dgetrf (partial pivoting) + dgetri.
 * erfinv is computed through Wichura's AS241 (PPND16) normal quantile.
 */
#include "sglm_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------- */
/* Normal distribution helpers (Breeze Gaussian(0,1))                          */
/* ------------------------------------------------------------------------- */

/* AS241 PPND16: normal quantile, ~1e-16 relative accuracy. */
static double ppnd16(double p) {
  double q = p - 0.5, r, val;
  if (fabs(q) <= 0.425) {
    r = 0.180625 - q * q;
    return q * (((((((2.5090809287301226727e+3 * r + 3.3430575583588128105e+4) * r +
                      6.7265770927008700853e+4) * r + 4.5921953931549871457e+4) * r +
                    1.3731693765509461125e+4) * r + 1.9715909503065514427e+3) * r +
                  1.3314166789178437745e+2) * r + 3.3871328727963666080e+0) /
           (((((((5.2264952788528545610e+3 * r + 2.8729085735721942674e+4) * r +
                 3.9307895800092710610e+4) * r + 2.1213794301586595867e+4) * r +
               5.3941960214247511077e+3) * r + 6.8718700749205790830e+2) * r +
             4.2313330701600911252e+1) * r + 1.0);
  }
  r = q < 0 ? p : 1.0 - p;
  if (r <= 0) return q < 0 ? -INFINITY : INFINITY;
  r = sqrt(-log(r));
  if (r <= 5.0) {
    r -= 1.6;
    val = (((((((7.74545014278341407640e-4 * r + 2.27238449892691845833e-2) * r +
                2.41780725177450611770e-1) * r + 1.27045825245236838258e+0) * r +
              3.64784832476320460504e+0) * r + 5.76949722146069140550e+0) * r +
            4.63033784615654529590e+0) * r + 1.42343711074968357734e+0) /
          (((((((1.05075007164441684324e-9 * r + 5.47593808499534494600e-4) * r +
                1.51986665636164571966e-2) * r + 1.48103976427480074590e-1) * r +
              6.89767334985100004550e-1) * r + 1.67638483018380384940e+0) * r +
            2.05319162663775882187e+0) * r + 1.0);
  } else {
    r -= 5.0;
    val = (((((((2.01033439929228813265e-7 * r + 2.71155556874348757815e-5) * r +
                1.24266094738807843860e-3) * r + 2.65321895265761230930e-2) * r +
              2.96560571828504891230e-1) * r + 1.78482653991729133580e+0) * r +
            5.46378491116411436990e+0) * r + 6.65790464350110377720e+0) /
          (((((((2.04426310338993978564e-15 * r + 1.42151175831644588870e-7) * r +
                1.84631831751005468180e-5) * r + 7.86869131145613259100e-4) * r +
              1.48753612908506148525e-2) * r + 1.36929880922735805310e-1) * r +
            5.99832206555887937690e-1) * r + 1.0);
  }
  return q < 0 ? -val : val;
}

double orc_erfinv(double x) {
  if (x <= -1.0) return x == -1.0 ? -INFINITY : NAN;
  if (x >= 1.0) return x == 1.0 ? INFINITY : NAN;
  return ppnd16((x + 1.0) / 2.0) / sqrt(2.0);
}

/* Breeze Gaussian(0,1).cdf, used by unlinkProbit (GLM.scala:231) */
double orc_norm_cdf(double x) { return 0.5 * (1.0 + erf(x / sqrt(2.0))); }

/* Breeze Gaussian(0,1).icdf, used by linkProbit (GLM.scala:212) */
double orc_norm_icdf(double q) { return 0.0 + 1.0 * sqrt(2.0) * orc_erfinv(2.0 * q - 1.0); }

/* Breeze Gaussian(0,1).pdf, used by lPrimeProbit (GLM.scala:222) */
static double norm_pdf(double x) {
  double d = (x - 0.0) / 1.0;
  return exp(-d * d / 2.0 - (log(sqrt(2.0 * M_PI)) + log(1.0)));
}

/* ------------------------------------------------------------------------- */
/* Family / link elementwise math (GLM.scala:90-251; extension families: R)   */
/* ------------------------------------------------------------------------- */

static double link_fn(int family, int link, double mu, double m) {
  if (family == ORC_BINOMIAL) {
    if (link == ORC_LOGIT) return log(mu / (m + (-1.0 * mu)));                 /* GLM.scala:193 */
    if (link == ORC_PROBIT) return orc_norm_icdf(mu / m);                       /* GLM.scala:212 */
    return log(-1.0 * log(1.0 + (-1.0 * (mu / m))));                            /* GLM.scala:240 */
  }
  if (family == ORC_GAUSSIAN) return mu;
  if (family == ORC_POISSON) return log(mu);
  return 1.0 / mu; /* gamma / inverse */
}

static double unlink_fn(int family, int link, double eta, double m) {
  if (family == ORC_BINOMIAL) {
    if (link == ORC_LOGIT) return m / (1.0 + exp(-1.0 * eta));                   /* GLM.scala:203 */
    if (link == ORC_PROBIT) return m * orc_norm_cdf(eta);                         /* GLM.scala:231 */
    return m * (1.0 + (-1.0 * exp(-exp(eta))));                                  /* GLM.scala:250 */
  }
  if (family == ORC_GAUSSIAN) return eta;
  if (family == ORC_POISSON) return exp(eta);
  return 1.0 / eta;
}

static double lprime_fn(int family, int link, double mu, double m) {
  if (family == ORC_BINOMIAL) {
    if (link == ORC_LOGIT) return m / (mu * (m + (-1.0 * mu)));                  /* GLM.scala:198 */
    if (link == ORC_PROBIT) return 1.0 / (m * norm_pdf(orc_norm_icdf(mu / m)));   /* GLM.scala:219-222 */
    return 1.0 / ((mu + (-1.0 * m)) * log(1.0 + (-1.0 * (mu / m))));             /* GLM.scala:245 */
  }
  if (family == ORC_GAUSSIAN) return 1.0;
  if (family == ORC_POISSON) return 1.0 / mu;
  return -1.0 / (mu * mu);
}

static double variance_fn(int family, double mu, double m) {
  if (family == ORC_BINOMIAL) return mu * (1.0 + (-1.0 * (mu / m)));            /* GLM.scala:128 */
  if (family == ORC_GAUSSIAN) return 1.0;
  if (family == ORC_POISSON) return mu;
  return mu * mu;
}

/* Breeze Binomial(n, p).logProbabilityOf(k) (called at GLM.scala:140 with p = mu). */
static double binom_logpmf(double mval, double mu, double yval, int *bad) {
  int n = (int)mval, k = (int)yval; /* .toInt truncation, GLM.scala:140 */
  if (n <= 0 || k < 0 || k > n || mu < 0.0) { *bad += 1; return NAN; }
  if (mu == 0.0) return k == 0 ? 0.0 : -INFINITY;
  if (mu == 1.0) return k == n ? 0.0 : -INFINITY;
  return lgamma(n + 1.0) - lgamma(k + 1.0) - lgamma(n - k + 1.0) + k * log(mu) + (n - k) * log1p(-mu);
}

/* Per-row unit contributions.  dev_i follows devBinomial's row value (GLM.scala:166-167);
 * the family factor (2 for binomial/poisson/gamma, 1 for gaussian) is applied after summing. */
static double unit_dev(int family, double y, double mu, double m, double pw) {
  if (family == ORC_BINOMIAL) {
    double my = m + (-1.0 * y);
    return pw * ((y * log(fmax(y, 1.0) / mu)) + (my * log(fmax(my, 1.0) / (m + (-1.0 * mu)))));
  }
  if (family == ORC_GAUSSIAN) { double r = y - mu; return pw * (r * r); }
  if (family == ORC_POISSON) return pw * ((y > 0.0 ? y * log(y / mu) : 0.0) - (y - mu));
  return pw * (-(log(y / mu) - (y - mu) / mu));
}

static double family_dev_factor(int family) { return family == ORC_GAUSSIAN ? 1.0 : 2.0; }

/* ------------------------------------------------------------------------- */
/* Summation: blocked pairwise (deterministic, ~log2(n) ulp error growth)      */
/* ------------------------------------------------------------------------- */
static double pairwise_sum(const double *v, int64_t n) {
  if (n <= 64) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += v[i];
    return s;
  }
  int64_t h = n / 2;
  return pairwise_sum(v, h) + pairwise_sum(v + h, n - h);
}

/* ------------------------------------------------------------------------- */
/* Gramian X'WX (lower) and X'Wz over rows [r0,r1): utils.scala:68-92           */
/* ------------------------------------------------------------------------- */
#define ORC_RB 256
static void gram_rows(const double *X, int64_t ldx, int64_t p, int64_t r0, int64_t r1,
                      const double *w, const double *z, double *G /* p*p col-major, lower */,
                      double *xtwz) {
  double *xw = (double *)malloc(sizeof(double) * ORC_RB * (size_t)p);
  for (int64_t c0 = r0; c0 < r1; c0 += ORC_RB) {
    int64_t nb = (r1 - c0) < ORC_RB ? (r1 - c0) : ORC_RB;
    /* leftMultDiag: XtW (utils.scala:68-80), kept in a chunk buffer */
    for (int64_t j = 0; j < p; ++j) {
      const double *xc = X + j * ldx + c0;
      double *o = xw + j * ORC_RB;
      for (int64_t r = 0; r < nb; ++r) o[r] = xc[r] * w[c0 + r];
    }
    /* XtW * X (utils.scala:89) -- lower triangle, 2x2 register blocks */
    for (int64_t j = 0; j < p; j += 2) {
      for (int64_t i = j; i < p; i += 2) {
        int64_t i1 = i + 1 < p ? i + 1 : i, j1 = j + 1 < p ? j + 1 : j;
        const double *a0 = X + i * ldx + c0, *a1 = X + i1 * ldx + c0;
        const double *b0 = xw + j * ORC_RB, *b1 = xw + j1 * ORC_RB;
        double s00 = 0, s01 = 0, s10 = 0, s11 = 0;
#pragma omp simd reduction(+ : s00, s01, s10, s11)
        for (int64_t r = 0; r < nb; ++r) {
          s00 += a0[r] * b0[r];
          s01 += a0[r] * b1[r];
          s10 += a1[r] * b0[r];
          s11 += a1[r] * b1[r];
        }
        G[i + j * p] += s00;
        if (j1 != j && i >= j1) G[i + j1 * p] += s01;
        if (i1 != i) {
          G[i1 + j * p] += s10;
          if (j1 != j) G[i1 + j1 * p] += s11;
        }
      }
    }
    /* XtW * y (utils.scala:90) */
    for (int64_t j = 0; j < p; ++j) {
      const double *b = xw + j * ORC_RB;
      double s = 0;
#pragma omp simd reduction(+ : s)
      for (int64_t r = 0; r < nb; ++r) s += b[r] * z[c0 + r];
      xtwz[j] += s;
    }
  }
  free(xw);
}

static void symmetrize_lower(double *G, int64_t p) {
  for (int64_t j = 0; j < p; ++j)
    for (int64_t i = j + 1; i < p; ++i) G[j + i * p] = G[i + j * p];
}

/* ------------------------------------------------------------------------- */
/* Breeze inv(): dgetrf + dgetri semantics (utils.scala:103, 134; LM.scala:197,225) */
/* ------------------------------------------------------------------------- */
int orc_lu_inverse(double *A, int64_t p) {
  int64_t *piv = (int64_t *)malloc(sizeof(int64_t) * (size_t)p);
  /* dgetrf: unblocked right-looking LU with partial pivoting */
  for (int64_t k = 0; k < p; ++k) {
    int64_t ip = k;
    double amax = fabs(A[k + k * p]);
    for (int64_t i = k + 1; i < p; ++i)
      if (fabs(A[i + k * p]) > amax) { amax = fabs(A[i + k * p]); ip = i; }
    piv[k] = ip;
    if (A[ip + k * p] == 0.0) { free(piv); return ORC_ESINGULAR; } /* MatrixSingularException */
    if (ip != k)
      for (int64_t j = 0; j < p; ++j) { double t = A[k + j * p]; A[k + j * p] = A[ip + j * p]; A[ip + j * p] = t; }
    double inv = 1.0 / A[k + k * p];
    for (int64_t i = k + 1; i < p; ++i) A[i + k * p] *= inv;
    for (int64_t j = k + 1; j < p; ++j) {
      double a = A[k + j * p];
      if (a != 0.0)
        for (int64_t i = k + 1; i < p; ++i) A[i + j * p] -= A[i + k * p] * a;
    }
  }
  /* dgetri step 1: inv(U) in place (dtrtri, upper, non-unit) */
  for (int64_t j = 0; j < p; ++j) {
    A[j + j * p] = 1.0 / A[j + j * p];
    double ajj = -A[j + j * p];
    /* compute elements 0..j-1 of column j: x = inv(U[0:j,0:j]) * U[0:j,j] (dtrmv) */
    for (int64_t k = 0; k < j; ++k) {
      double t = A[k + j * p];
      if (t != 0.0) {
        for (int64_t i = 0; i < k; ++i) A[i + j * p] += t * A[i + k * p];
        A[k + j * p] = t * A[k + k * p];
      }
    }
    for (int64_t i = 0; i < j; ++i) A[i + j * p] *= ajj;
  }
  /* dgetri step 2: solve inv(A)*L = inv(U) for inv(A), columns right to left */
  double *work = (double *)malloc(sizeof(double) * (size_t)p);
  for (int64_t j = p - 1; j >= 0; --j) {
    for (int64_t i = j + 1; i < p; ++i) { work[i] = A[i + j * p]; A[i + j * p] = 0.0; }
    for (int64_t k = j + 1; k < p; ++k) {
      double t = work[k];
      if (t != 0.0)
        for (int64_t i = 0; i < p; ++i) A[i + j * p] -= A[i + k * p] * t;
    }
  }
  /* apply column interchanges in reverse */
  for (int64_t j = p - 2; j >= 0; --j) {
    int64_t jp = piv[j];
    if (jp != j)
      for (int64_t i = 0; i < p; ++i) { double t = A[i + j * p]; A[i + j * p] = A[i + jp * p]; A[i + jp * p] = t; }
  }
  free(work);
  free(piv);
  return ORC_OK;
}

/* wlsSingle / wlsMultiple tail (utils.scala:103-106, 134-137):
 * XtWXi = inv(XtWX); coefs = XtWXi * XtWy; diagDesign = sqrt(diag(XtWXi)) */
static int wls_solve(double *G /* full p*p, destroyed -> inverse */, const double *xtwz, int64_t p,
                     double *coefs, double *diag_design) {
  int rc = orc_lu_inverse(G, p);
  if (rc) return rc;
  for (int64_t i = 0; i < p; ++i) {
    double s = 0.0;
    for (int64_t k = 0; k < p; ++k) s += G[i + k * p] * xtwz[k];
    coefs[i] = s;
    diag_design[i] = sqrt(G[i + i * p]);
  }
  return ORC_OK;
}

/* ------------------------------------------------------------------------- */
/* Partition helpers (Spark ParallelCollectionRDD slicing: [i*n/G, (i+1)*n/G)) */
/* ------------------------------------------------------------------------- */
static int64_t part_lo(int64_t n, int g, int G) { return (int64_t)(((__int128)g * n) / G); }

typedef struct {
  const double *X; int64_t n, p, ldx;
  const double *y, *m, *offset, *prior;
  int family, link;
} orc_data;

static inline double M_(const orc_data *d, int64_t i) { return d->m ? d->m[i] : 1.0; }
static inline double OFF_(const orc_data *d, int64_t i) { return d->offset ? d->offset[i] : 0.0; }
static inline double PW_(const orc_data *d, int64_t i) { return d->prior ? d->prior[i] : 1.0; }

/* eta = X*coefs + offset (GLM.scala:292 single; etaCreate :321-332 multiple) */
static void eta_create(const orc_data *d, const double *coefs, double *eta, int add_offset) {
  for (int64_t i = 0; i < d->n; ++i) eta[i] = 0.0;
  for (int64_t j = 0; j < d->p; ++j) {
    const double *xc = d->X + j * d->ldx;
    double b = coefs[j];
    for (int64_t i = 0; i < d->n; ++i) eta[i] += xc[i] * b;
  }
  if (add_offset)
    for (int64_t i = 0; i < d->n; ++i) eta[i] = eta[i] + OFF_(d, i);
}

/* Deviance over rows [a,b): devBinomial (GLM.scala:162-170) for one partition. */
static double dev_range(const orc_data *d, const double *mu, int64_t a, int64_t b, double *tmp) {
  for (int64_t i = a; i < b; ++i) tmp[i - a] = unit_dev(d->family, d->y[i], mu[i], M_(d, i), PW_(d, i));
  return family_dev_factor(d->family) * pairwise_sum(tmp, b - a);
}

/* createBinomialDeviance (GLM.scala:397-408): per-partition deviance summed in partition order */
static double dev_total(const orc_data *d, const double *mu, int G, double *tmp) {
  double s = 0.0;
  for (int g = 0; g < G; ++g) s += dev_range(d, mu, part_lo(d->n, g, G), part_lo(d->n, g + 1, G), tmp);
  return s;
}

/* Gram over all partitions with a tree reduction (wlsComponents, utils.scala:110-126) */
static void gram_partitioned(const orc_data *d, const double *w, const double *z, int G, int nthreads,
                             double *Gout, double *xtwz_out) {
  int64_t p = d->p;
  double *parts = (double *)calloc((size_t)G * (size_t)(p * p + p), sizeof(double));
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
  for (int g = 0; g < G; ++g) {
    double *Gg = parts + (size_t)g * (size_t)(p * p + p);
    gram_rows(d->X, d->ldx, p, part_lo(d->n, g, G), part_lo(d->n, g + 1, G), w, z, Gg, Gg + p * p);
  }
  (void)nthreads;
  /* treeReduce(reduceNormal): pairwise tree, deterministic order */
  for (int step = 1; step < G; step *= 2)
    for (int g = 0; g + step < G; g += 2 * step) {
      double *a = parts + (size_t)g * (size_t)(p * p + p), *b = parts + (size_t)(g + step) * (size_t)(p * p + p);
      for (int64_t k = 0; k < p * p + p; ++k) a[k] += b[k];
    }
  memcpy(Gout, parts, sizeof(double) * (size_t)(p * p));
  memcpy(xtwz_out, parts + p * p, sizeof(double) * (size_t)p);
  symmetrize_lower(Gout, p);
  free(parts);
}

/* Final statistics over rows (pearsonCalc GLM.scala:90-118; llBinomial :132-159). */
static void final_stats(const orc_data *d, const double *mu, int G, double dev, double *pearson,
                        double *ll, int *bad, double *tmp) {
  int64_t n = d->n;
  double pear = 0.0, lls = 0.0;
  for (int g = 0; g < G; ++g) {
    int64_t a = part_lo(n, g, G), b = part_lo(n, g + 1, G);
    /* pearsonCalc: binomial variance regardless of family in the reference (GLM.scala:95-99);
       the extension families use their own variance. */
    for (int64_t i = a; i < b; ++i) {
      double r = d->y[i] + (-1.0 * mu[i]);
      tmp[i - a] = PW_(d, i) * (r * r) / variance_fn(d->family, mu[i], M_(d, i));
    }
    pear += pairwise_sum(tmp, b - a);
    if (d->family == ORC_BINOMIAL) {
      for (int64_t i = a; i < b; ++i) tmp[i - a] = PW_(d, i) * binom_logpmf(M_(d, i), mu[i], d->y[i], bad);
      lls += pairwise_sum(tmp, b - a);
    } else if (d->family == ORC_POISSON) {
      for (int64_t i = a; i < b; ++i)
        tmp[i - a] = PW_(d, i) * (d->y[i] * log(mu[i]) - mu[i] - lgamma(d->y[i] + 1.0));
      lls += pairwise_sum(tmp, b - a);
    }
  }
  if (d->family == ORC_GAUSSIAN) {
    /* R gaussian()$aic with sigma^2 = dev/n: ll = -(n/2)(log(2 pi dev/n)+1) + 0.5*sum(log w) */
    double slw = 0.0;
    if (d->prior) { for (int64_t i = 0; i < n; ++i) tmp[i] = log(d->prior[i]); slw = pairwise_sum(tmp, n); }
    lls = -((double)n / 2.0) * (log(2.0 * M_PI * dev / (double)n) + 1.0) + 0.5 * slw;
  } else if (d->family == ORC_GAMMA) {
    /* R Gamma()$aic: disp = dev/sum(w); ll = sum w*dgamma(y, 1/disp, scale=mu*disp, log) */
    double sw = 0, swly = 0, swymu = 0, swlmu = 0;
    for (int64_t i = 0; i < n; ++i) tmp[i] = PW_(d, i);
    sw = pairwise_sum(tmp, n);
    for (int64_t i = 0; i < n; ++i) tmp[i] = PW_(d, i) * log(d->y[i]);
    swly = pairwise_sum(tmp, n);
    for (int64_t i = 0; i < n; ++i) tmp[i] = PW_(d, i) * (d->y[i] / mu[i]);
    swymu = pairwise_sum(tmp, n);
    for (int64_t i = 0; i < n; ++i) tmp[i] = PW_(d, i) * log(mu[i]);
    swlmu = pairwise_sum(tmp, n);
    double disp = dev / sw, a = 1.0 / disp;
    lls = (a - 1.0) * swly - swymu / disp - (lgamma(a) + a * log(disp)) * sw - a * swlmu;
  }
  *pearson = pear;
  *ll = lls;
}

/* ------------------------------------------------------------------------- */
/* The IRLS driver: fitSingleBinomial (G==1, GLM.scala:254-315) and           */
/* fitMultipleBinomial (G>1, GLM.scala:410-468).                               */
/* ------------------------------------------------------------------------- */
int orc_fit_glm(const double *X, int64_t n, int64_t p, int64_t ldx, const double *y, const double *m,
                const double *offset, const double *prior, const orc_opts *o, orc_preglm *out) {
  if (n <= 0 || p <= 0 || ldx < n) return ORC_EINVAL;
  orc_data d = {X, n, p, ldx, y, m, offset, prior, o->family, o->link};
  int G = o->npart > 0 ? o->npart : 1;
  double *mu = malloc(sizeof(double) * n), *eta = malloc(sizeof(double) * n);
  double *w = malloc(sizeof(double) * n), *z = malloc(sizeof(double) * n), *tmp = malloc(sizeof(double) * n);
  double *Gm = malloc(sizeof(double) * p * p), *xtwz = malloc(sizeof(double) * p);
  double *coefs = calloc(p, sizeof(double)), *diag_design = calloc(p, sizeof(double));
  int rc = ORC_OK;

  /* Initialize: mu = mean(y) (GLM.scala:263 single; :420-425 multiple: per-partition sums) */
  double ysum = 0.0;
  for (int g = 0; g < G; ++g) {
    int64_t a = part_lo(n, g, G), b = part_lo(n, g + 1, G);
    ysum += pairwise_sum(y + a, b - a);
  }
  double ymean = ysum / (double)n;
  for (int64_t i = 0; i < n; ++i) mu[i] = ymean;
  /* eta = link(mu, m), offset ignored (GLM.scala:264-270, 429-442) */
  for (int64_t i = 0; i < n; ++i) eta[i] = link_fn(o->family, o->link, mu[i], M_(&d, i));
  double dev = dev_total(&d, mu, G, tmp); /* GLM.scala:271 / 443 */
  double null_dev = dev, dev_old = dev, deltad = 1.0;
  int iter = 0;
  if (out->dev_trace && out->max_trace > 0) out->dev_trace[0] = dev;

  while (fabs(deltad) > o->tol) { /* GLM.scala:281 / 452 */
    if (o->max_iter > 0 && iter >= o->max_iter) break;
    /* G==1: grad from the stored mu (GLM.scala:282-290).
       G>1: zwCreateBinomial re-derives mu = unlink(eta) (GLM.scala:370-371). */
    for (int64_t i = 0; i < n; ++i) {
      double mi = M_(&d, i);
      double mui = (G == 1) ? mu[i] : unlink_fn(o->family, o->link, eta[i], mi);
      double grad = lprime_fn(o->family, o->link, mui, mi);
      w[i] = PW_(&d, i) * (1.0 / (variance_fn(o->family, mui, mi) * (grad * grad)));
      z[i] = (eta[i] + ((y[i] + (-1.0 * mui)) * grad)) + (-1.0 * OFF_(&d, i));
    }
    gram_partitioned(&d, w, z, G, o->nthreads, Gm, xtwz);
    rc = wls_solve(Gm, xtwz, p, coefs, diag_design);
    if (rc) goto done;
    eta_create(&d, coefs, eta, 1);
    for (int64_t i = 0; i < n; ++i) mu[i] = unlink_fn(o->family, o->link, eta[i], M_(&d, i));
    dev_old = dev;
    dev = dev_total(&d, mu, G, tmp);
    deltad = dev - dev_old;
    iter = iter + 1;
    if (out->dev_trace && iter < out->max_trace) out->dev_trace[iter] = dev;
    if (o->verbose) printf("%d\t%.17g\n", iter, deltad);
  }
  {
    int bad = 0;
    double pearson, ll;
    final_stats(&d, mu, G, dev, &pearson, &ll, &bad, tmp);
    if (bad) { rc = ORC_EINVAL; goto done; }
    memcpy(out->coefs, coefs, sizeof(double) * p);
    memcpy(out->stderr_, diag_design, sizeof(double) * p);
    out->deviance = dev;
    out->null_deviance = null_dev;
    out->pearson = pearson;
    out->loglik = ll;
    out->iter = iter;
    out->nrow = (double)n;
    out->npart = G;
  }
done:
  free(mu); free(eta); free(w); free(z); free(tmp); free(Gm); free(xtwz); free(coefs); free(diag_design);
  return rc;
}

/* ------------------------------------------------------------------------- */
/* LM (LM.scala:142-274)                                                       */
/* ------------------------------------------------------------------------- */
int orc_fit_lm(const double *X, int64_t n, int64_t p, int64_t ldx, const double *y, int npart, int nthreads,
               double *coefs, double *xtxi, double *stderr_, double *sse_o, double *r2_o, double *fstat_o,
               double *sigma_o) {
  if (n <= 0 || p <= 0 || ldx < n) return ORC_EINVAL;
  int G = npart > 0 ? npart : 1;
  orc_data d = {X, n, p, ldx, y, NULL, NULL, NULL, ORC_GAUSSIAN, ORC_IDENTITY};
  double *ones = malloc(sizeof(double) * n), *xty = malloc(sizeof(double) * p), *pred = malloc(sizeof(double) * n);
  double *tmp = malloc(sizeof(double) * n);
  for (int64_t i = 0; i < n; ++i) ones[i] = 1.0;
  /* rowPartitionedComponents (LM.scala:142-155) / fitSingle xm.t*xm (LM.scala:197-198) */
  gram_partitioned(&d, ones, y, G, nthreads, xtxi, xty);
  int rc = orc_lu_inverse(xtxi, p);
  if (rc) goto done;
  for (int64_t i = 0; i < p; ++i) {
    double s = 0.0;
    for (int64_t k = 0; k < p; ++k) s += xtxi[i + k * p] * xty[k];
    coefs[i] = s; /* LM.scala:199 / 227 */
  }
  eta_create(&d, coefs, pred, 0);
  /* rowPartitionedSSE (LM.scala:160-188): yMean then per-partition (sse, top, bot) */
  double ysum = 0.0;
  for (int g = 0; g < G; ++g) ysum += pairwise_sum(y + part_lo(n, g, G), part_lo(n, g + 1, G) - part_lo(n, g, G));
  double ymean = ysum / (double)n;
  double sse = 0, top = 0, bot = 0;
  for (int g = 0; g < G; ++g) {
    int64_t a = part_lo(n, g, G), b = part_lo(n, g + 1, G);
    for (int64_t i = a; i < b; ++i) { double e = y[i] - pred[i]; tmp[i - a] = e * e; }
    sse += pairwise_sum(tmp, b - a);
    for (int64_t i = a; i < b; ++i) { double e = pred[i] + (-1.0 * ymean); tmp[i - a] = e * e; }
    top += pairwise_sum(tmp, b - a);
    for (int64_t i = a; i < b; ++i) { double e = y[i] + (-1.0 * ymean); tmp[i - a] = e * e; }
    bot += pairwise_sum(tmp, b - a);
  }
  double r2 = top / bot;
  double fstat = ((bot - sse) / ((double)p - 1.0)) / (sse / ((double)n - (double)p));
  /* LM.fit (LM.scala:260-263) */
  double sig2 = sse / ((double)n - (double)p);
  for (int64_t i = 0; i < p; ++i) stderr_[i] = sqrt(sig2 * xtxi[i + i * p]);
  *sse_o = sse; *r2_o = r2; *fstat_o = fstat; *sigma_o = sqrt(sig2);
done:
  free(ones); free(xty); free(pred); free(tmp);
  return rc;
}

/* ------------------------------------------------------------------------- */
/* Shard partials in the engine's packed wire format (for distributed tests)   */
/* ------------------------------------------------------------------------- */
int orc_shard_partials(const double *X, int64_t n, int64_t p, int64_t ldx, const double *y, const double *m,
                       const double *offset, const double *prior, int family, int link, int mode,
                       const double *beta, double mu0, double ybar, double *packed) {
  if (n < 0 || p <= 0 || ldx < n) return ORC_EINVAL;
  orc_data d = {X, n, p, ldx, y, m, offset, prior, family, link};
  int64_t tri = p * (p + 1) / 2;
  memset(packed, 0, sizeof(double) * (size_t)(tri + p + ORC_NS));
  if (n == 0) return ORC_OK;
  double *s = packed + tri + p;
  double *eta = malloc(sizeof(double) * n), *mu = malloc(sizeof(double) * n);
  double *w = malloc(sizeof(double) * n), *z = malloc(sizeof(double) * n), *tmp = malloc(sizeof(double) * n);
  double *Gm = calloc(p * p, sizeof(double)), *xtwz = calloc(p, sizeof(double));
  if (mode == ORC_MODE_LM_RESID) {
    /* rowPartitionedSSE (LM.scala:160-188) at beta with the global mean ybar */
    eta_create(&d, beta, eta, 0);
    for (int64_t i = 0; i < n; ++i) { double e = y[i] - eta[i]; tmp[i] = e * e; }
    s[ORC_S_DEV] = pairwise_sum(tmp, n);
    for (int64_t i = 0; i < n; ++i) { double e = eta[i] + (-1.0 * ybar); tmp[i] = e * e; }
    s[ORC_S_PEARSON] = pairwise_sum(tmp, n);
    for (int64_t i = 0; i < n; ++i) { double e = y[i] + (-1.0 * ybar); tmp[i] = e * e; }
    s[ORC_S_LL] = pairwise_sum(tmp, n);
    s[ORC_S_SUMW] = (double)n;
    goto out;
  }
  if (mode == ORC_MODE_LM_GRAM) {
    /* rowPartitionedComponents (LM.scala:142-155): X'X, X'y; plus sum y and rows */
    for (int64_t i = 0; i < n; ++i) { w[i] = 1.0; z[i] = y[i]; }
    gram_rows(X, ldx, p, 0, n, w, z, Gm, xtwz);
    s[ORC_S_DEV] = pairwise_sum(y, n);
    s[ORC_S_SUMW] = (double)n;
    goto pack;
  }
  if (mode == ORC_MODE_IRLS) {
    eta_create(&d, beta, eta, 1);
    for (int64_t i = 0; i < n; ++i) mu[i] = unlink_fn(family, link, eta[i], M_(&d, i));
  } else {
    for (int64_t i = 0; i < n; ++i) {
      eta[i] = link_fn(family, link, mu0, M_(&d, i));
      mu[i] = (mode == ORC_MODE_INIT_SINGLE) ? mu0 : unlink_fn(family, link, eta[i], M_(&d, i));
    }
  }
  for (int64_t i = 0; i < n; ++i) {
    double mi = M_(&d, i), grad = lprime_fn(family, link, mu[i], mi);
    w[i] = PW_(&d, i) * (1.0 / (variance_fn(family, mu[i], mi) * (grad * grad)));
    z[i] = (eta[i] + ((y[i] + (-1.0 * mu[i])) * grad)) + (-1.0 * OFF_(&d, i));
  }
  gram_rows(X, ldx, p, 0, n, w, z, Gm, xtwz);
  /* fitMultipleBinomial re-derives mu = unlink(link(ybar)) only inside zwCreateBinomial; the null
     deviance (and the statistics of a fit that stops before its first solve) are taken at
     mu0 = ybar itself (GLM.scala:424-444). */
  if (mode == ORC_MODE_INIT_MULTI)
    for (int64_t i = 0; i < n; ++i) mu[i] = mu0;
  for (int64_t i = 0; i < n; ++i) tmp[i] = unit_dev(family, y[i], mu[i], M_(&d, i), PW_(&d, i));
  s[ORC_S_DEV] = pairwise_sum(tmp, n);
  for (int64_t i = 0; i < n; ++i) {
    double r = y[i] + (-1.0 * mu[i]);
    tmp[i] = PW_(&d, i) * (r * r) / variance_fn(family, mu[i], M_(&d, i));
  }
  s[ORC_S_PEARSON] = pairwise_sum(tmp, n);
  {
    int bad = 0;
    if (family == ORC_BINOMIAL) {
      for (int64_t i = 0; i < n; ++i) tmp[i] = PW_(&d, i) * binom_logpmf(M_(&d, i), mu[i], y[i], &bad);
      s[ORC_S_LL] = pairwise_sum(tmp, n);
    } else if (family == ORC_POISSON) {
      for (int64_t i = 0; i < n; ++i) tmp[i] = PW_(&d, i) * (y[i] * log(mu[i]) - mu[i] - lgamma(y[i] + 1.0));
      s[ORC_S_LL] = pairwise_sum(tmp, n);
    } else if (family == ORC_GAUSSIAN) {
      for (int64_t i = 0; i < n; ++i) tmp[i] = log(PW_(&d, i));
      s[ORC_S_LL] = pairwise_sum(tmp, n);
    } else {
      for (int64_t i = 0; i < n; ++i) tmp[i] = PW_(&d, i) * log(y[i]);
      s[ORC_S_LL] = pairwise_sum(tmp, n);
      for (int64_t i = 0; i < n; ++i) tmp[i] = PW_(&d, i) * (y[i] / mu[i]);
      s[ORC_S_AUX0] = pairwise_sum(tmp, n);
      for (int64_t i = 0; i < n; ++i) tmp[i] = PW_(&d, i) * log(mu[i]);
      s[ORC_S_AUX1] = pairwise_sum(tmp, n);
    }
    s[ORC_S_BAD] = (double)bad;
  }
  for (int64_t i = 0; i < n; ++i) tmp[i] = PW_(&d, i);
  s[ORC_S_SUMW] = pairwise_sum(tmp, n);
pack:
  for (int64_t i = 0; i < p; ++i)
    for (int64_t j = 0; j <= i; ++j) packed[i * (i + 1) / 2 + j] = Gm[i + j * p];
  for (int64_t j = 0; j < p; ++j) packed[tri + j] = xtwz[j];
out:
  free(eta); free(mu); free(w); free(z); free(tmp); free(Gm); free(xtwz);
  return ORC_OK;
}

/* ------------------------------------------------------------------------- */
/* Streaming ("procedural") fits for designs larger than host RAM (SURVEY.md    */
/* 8(d): "for sizes beyond host RAM, regenerate rows on the fly from the same    */
/* generator").  The rows come from the seeded counter-based generator of       */
/* sparkglm_amd/synth.py (bit-identical: integer splitmix64, IEEE mul/add, no    */
/* contraction); every IRLS iteration regenerates them chunk by chunk, so only  */
/* p x p state is kept.  The fit is the single-pass restatement of               */
/* fitSingleBinomial (GLM.scala:254-315; npart > 1: fitMultipleBinomial's        */
/* mu = unlink(link(ybar)) first step, GLM.scala:370-371): pass k at beta_k      */
/* yields dev_k (the loop test, GLM.scala:301-303), pearson / loglik at mu_k     */
/* (GLM.scala:307-311) and X'W_kX, X'W_kz_k for the next wlsSingle solve         */
/* (utils.scala:98-107) -- the same quantities the reference derives from its    */
/* stored mu, since mu_k = unlink(X beta_k + offset).  Sums run in a fixed order */
/* (64 contiguous row segments, chunks in order inside each) independent of the  */
/* thread count.                                                                 */
/* ------------------------------------------------------------------------- */
static inline uint64_t sm64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static inline double unif64(uint64_t key) { return (double)(sm64(key) >> 11) * 0x1.0p-53; }

typedef struct {
  int kind;
  int64_t p;
  uint64_t kx, ky, ko, kp;
  double scale;
  double *bs; /* beta* of the generator */
} orc_gen;

static void gen_init(orc_gen *g, int kind, int64_t p, uint64_t seed) {
  g->kind = kind;
  g->p = p;
  g->kx = sm64(seed);
  g->ky = sm64(seed ^ 0x5555555555555555ULL);
  g->ko = sm64(seed ^ 0x3333333333333333ULL);
  g->kp = sm64(seed ^ 0x0F0F0F0F0F0F0F0FULL);
  g->scale = 1.0 / sqrt((double)p);
  g->bs = (double *)malloc(sizeof(double) * (size_t)p);
  for (int64_t j = 0; j < p; ++j) g->bs[j] = kind == 3 ? 0.1 * (double)((j % 5) + 1) : 0.5 * (double)((j % 5) - 2);
  g->bs[0] = kind == 3 ? 1.0 : -0.25;
}

/* Rows [gi0, gi0+nr) (global indices) into X (ld rows), y, offset / prior (kind 2). */
static void gen_rows(const orc_gen *g, int64_t gi0, int64_t nr, double *X, int64_t ld, double *y, double *off,
                     double *pr) {
  const int64_t p = g->p;
  for (int64_t i = 0; i < nr; ++i) {
    const uint64_t gi = (uint64_t)(gi0 + i);
    const uint64_t base = g->kx + gi * (uint64_t)p;
    double eta = 0.0;
    for (int64_t j = 0; j < p; ++j) {
      double x;
      if (j == 0) x = 1.0;
      else if (g->kind == 3) x = (0.5 + unif64(base + (uint64_t)j)) * g->scale;
      else x = (2.0 * unif64(base + (uint64_t)j) - 1.0) * g->scale;
      X[i + j * ld] = x;
      double prod = x * g->bs[j];
      eta = eta + prod;
    }
    const double u = unif64(g->ky + gi);
    if (off) off[i] = 0.0;
    if (pr) pr[i] = 1.0;
    if (g->kind == 0) {
      double q = fmin(fmax(0.5 + 0.25 * eta, 0.02), 0.98);
      y[i] = u < q ? 1.0 : 0.0;
    } else if (g->kind == 1) {
      y[i] = eta + (2.0 * u - 1.0);
    } else if (g->kind == 2) {
      double lam = fmax(1.0 + 0.5 * eta, 0.1);
      y[i] = floor(u * 2.0 * lam);
      if (off) off[i] = (2.0 * unif64(g->ko + gi) - 1.0) * 0.1;
      if (pr) pr[i] = 0.5 + unif64(g->kp + gi);
    } else {
      y[i] = (0.25 + 1.5 * u) / eta;
    }
  }
}

int orc_synth_rows(int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed, double *X, double *y, double *off,
                   double *pr) {
  if (kind < 0 || kind > 3 || n < 0 || p <= 0) return ORC_EINVAL;
  orc_gen g;
  gen_init(&g, kind, p, seed);
  gen_rows(&g, row0, n, X, n, y, off, pr);
  free(g.bs);
  return ORC_OK;
}

#define ORC_NSEG 64
#define ORC_CH 256

enum { SP_YSUM = 100 };

typedef struct {
  double *G, *xtwz; /* G: p*p col-major, lower triangle accumulated */
  double s[ORC_NS], c[ORC_NS]; /* scalar sums with Neumaier compensation terms */
} seg_acc;

/* Compensated (Neumaier) accumulation: at 1e9 rows a plain running sum of the deviance carries
 * ~1e-6 of rounding noise -- the size of GLM.scala:281's absolute tol -- so the iteration count
 * would follow the summation order instead of the fit.  The compensated sum is accurate to
 * about one ulp of the total. */
static inline void neumaier(double *s, double *c, double x) {
  double t = *s + x;
  if (fabs(*s) >= fabs(x)) *c += (*s - t) + x;
  else *c += (x - t) + *s;
  *s = t;
}

/* One pass over rows [row0, row0+n) of the generated design (see the section comment).
 * nseg > 0 (plain_sums): nseg contiguous partitions, each one thread's, its scalars a plain
 * running sum over its rows in row order (reference BLAS's ones-vector dgemm, GLM.scala:168). */
static void stream_pass(const orc_gen *g, int64_t row0, int64_t n, int family, int link, int mode,
                        const double *beta, double mu0, int nthreads, seg_acc *seg, int nseg) {
  const int plain = nseg > 0;
  if (!plain) nseg = ORC_NSEG;
  const int64_t p = g->p;
  const int has_op = g->kind == 2;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
#endif
  {
    double *X = (double *)malloc(sizeof(double) * ORC_CH * (size_t)p);
    double *y = (double *)malloc(sizeof(double) * ORC_CH), *off = (double *)malloc(sizeof(double) * ORC_CH);
    double *pr = (double *)malloc(sizeof(double) * ORC_CH), *w = (double *)malloc(sizeof(double) * ORC_CH);
    double *z = (double *)malloc(sizeof(double) * ORC_CH), *t = (double *)malloc(sizeof(double) * ORC_CH * ORC_NS);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
    for (int sgi = 0; sgi < nseg; ++sgi) {
      seg_acc *a = &seg[sgi];
      memset(a->s, 0, sizeof a->s);
      memset(a->c, 0, sizeof a->c);
      if (mode != SP_YSUM) {
        memset(a->G, 0, sizeof(double) * (size_t)(p * p));
        memset(a->xtwz, 0, sizeof(double) * (size_t)p);
      }
      const int64_t lo = part_lo(n, sgi, nseg), hi = part_lo(n, sgi + 1, nseg);
      for (int64_t c0 = lo; c0 < hi; c0 += ORC_CH) {
        const int64_t nr = (hi - c0) < ORC_CH ? (hi - c0) : ORC_CH;
        gen_rows(g, row0 + c0, nr, X, ORC_CH, y, has_op ? off : NULL, has_op ? pr : NULL);
        if (mode == SP_YSUM) {
          if (plain)
            for (int64_t i = 0; i < nr; ++i) a->s[ORC_S_DEV] += y[i];
          else
            neumaier(&a->s[ORC_S_DEV], &a->c[ORC_S_DEV], pairwise_sum(y, nr));
          continue;
        }
        for (int64_t i = 0; i < nr; ++i) {
          const double oi = has_op ? off[i] : 0.0, pw = has_op ? pr[i] : 1.0;
          double eta, mu, mud;
          if (mode == ORC_MODE_IRLS) {
            eta = 0.0; /* eta_create (GLM.scala:292 / 321-332) */
            for (int64_t j = 0; j < p; ++j) eta += X[i + j * ORC_CH] * beta[j];
            eta = eta + oi;
            mu = unlink_fn(family, link, eta, 1.0);
            mud = mu;
          } else { /* eta = link(mu0), offset ignored (GLM.scala:264-270, 429-442) */
            eta = link_fn(family, link, mu0, 1.0);
            mu = (mode == ORC_MODE_INIT_SINGLE) ? mu0 : unlink_fn(family, link, eta, 1.0);
            mud = mu0; /* the null deviance is taken at mu0 itself (GLM.scala:271, 443) */
          }
          const double grad = lprime_fn(family, link, mu, 1.0);
          w[i] = pw * (1.0 / (variance_fn(family, mu, 1.0) * (grad * grad)));
          z[i] = (eta + ((y[i] + (-1.0 * mu)) * grad)) + (-1.0 * oi);
          const double r = y[i] + (-1.0 * mud);
          double *ti = t + i;
          ti[ORC_S_DEV * ORC_CH] = unit_dev(family, y[i], mud, 1.0, pw);
          ti[ORC_S_PEARSON * ORC_CH] = pw * (r * r) / variance_fn(family, mud, 1.0);
          ti[ORC_S_AUX0 * ORC_CH] = 0.0;
          ti[ORC_S_AUX1 * ORC_CH] = 0.0;
          ti[ORC_S_BAD * ORC_CH] = 0.0;
          if (family == ORC_BINOMIAL) {
            int bad = 0; /* m = 1: Binomial(1, mu).logProbabilityOf(y.toInt) (GLM.scala:140) */
            ti[ORC_S_LL * ORC_CH] = pw * binom_logpmf(1.0, mud, y[i], &bad);
            ti[ORC_S_BAD * ORC_CH] = (double)bad;
          } else if (family == ORC_POISSON) {
            ti[ORC_S_LL * ORC_CH] = pw * (y[i] * log(mud) - mud - lgamma(y[i] + 1.0));
          } else if (family == ORC_GAUSSIAN) {
            ti[ORC_S_LL * ORC_CH] = log(pw);
          } else {
            ti[ORC_S_LL * ORC_CH] = pw * log(y[i]);
            ti[ORC_S_AUX0 * ORC_CH] = pw * (y[i] / mud);
            ti[ORC_S_AUX1 * ORC_CH] = pw * log(mud);
          }
          ti[ORC_S_SUMW * ORC_CH] = pw;
        }
        for (int k = 0; k < ORC_NS; ++k) {
          if (k == ORC_S_AUX2) continue;
          if (plain)
            for (int64_t i = 0; i < nr; ++i) a->s[k] += t[k * ORC_CH + i];
          else
            neumaier(&a->s[k], &a->c[k], pairwise_sum(t + k * ORC_CH, nr));
        }
        gram_rows(X, ORC_CH, p, 0, nr, w, z, a->G, a->xtwz);
      }
    }
    free(X); free(y); free(off); free(pr); free(w); free(z); free(t);
  }
}

/* nseg > 0: plain_sums -- the partition totals added plainly in partition order (GLM.scala:407) */
static void seg_total(const seg_acc *seg, int64_t p, int with_gram, double *G, double *xtwz, double *s, int nseg) {
  double cs[ORC_NS] = {0};
  const int plain = nseg > 0;
  if (!plain) nseg = ORC_NSEG;
  memset(s, 0, sizeof(double) * ORC_NS);
  if (with_gram) {
    memset(G, 0, sizeof(double) * (size_t)(p * p));
    memset(xtwz, 0, sizeof(double) * (size_t)p);
  }
  for (int sgi = 0; sgi < nseg; ++sgi) {
    for (int k = 0; k < ORC_NS; ++k) {
      if (plain) {
        s[k] += seg[sgi].s[k];
        continue;
      }
      neumaier(&s[k], &cs[k], seg[sgi].s[k]);
      neumaier(&s[k], &cs[k], seg[sgi].c[k]);
    }
    if (!with_gram) continue;
    for (int64_t j = 0; j < p; ++j)
      for (int64_t i = j; i < p; ++i) G[i + j * p] += seg[sgi].G[i + j * p];
    for (int64_t j = 0; j < p; ++j) xtwz[j] += seg[sgi].xtwz[j];
  }
  for (int k = 0; k < ORC_NS; ++k) s[k] += cs[k];
  if (with_gram) symmetrize_lower(G, p);
}

/* One streaming pass of orc_fit_glm_synth at beta (its IRLS passes, GLM.scala:453-458 over the
 * generated rows): X'WX (p*p col-major, symmetric), X'Wz and the 8 scalars, summed exactly as the
 * fit sums them.  For comparing the engine's Gram with the oracle's at the same beta. */
int orc_pass_synth(int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed, int family, int link, int mode,
                   const double *beta, double mu0, int nthreads, double *G, double *xtwz, double *s) {
  if (kind < 0 || kind > 3 || n <= 0 || p <= 0 || !G || !xtwz || !s) return ORC_EINVAL;
  if (mode == ORC_MODE_IRLS && !beta) return ORC_EINVAL;
  orc_gen g;
  gen_init(&g, kind, p, seed);
  seg_acc *seg = (seg_acc *)calloc(ORC_NSEG, sizeof(seg_acc));
  for (int sgi = 0; sgi < ORC_NSEG; ++sgi) {
    seg[sgi].G = (double *)calloc((size_t)(p * p), sizeof(double));
    seg[sgi].xtwz = (double *)calloc((size_t)p, sizeof(double));
  }
  stream_pass(&g, row0, n, family, link, mode, beta, mu0, nthreads, seg, 0);
  seg_total(seg, p, 1, G, xtwz, s, 0);
  for (int sgi = 0; sgi < ORC_NSEG; ++sgi) { free(seg[sgi].G); free(seg[sgi].xtwz); }
  free(seg);
  free(g.bs);
  return ORC_OK;
}

int orc_fit_glm_synth(int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed, const orc_opts *o,
                      orc_preglm *out) {
  if (kind < 0 || kind > 3 || n <= 0 || p <= 0) return ORC_EINVAL;
  orc_gen g;
  gen_init(&g, kind, p, seed);
  const int nseg = o->plain_sums ? (o->npart > 0 ? o->npart : 1) : 0, nalloc = nseg > ORC_NSEG ? nseg : ORC_NSEG;
  seg_acc *seg = (seg_acc *)calloc((size_t)nalloc, sizeof(seg_acc));
  for (int sgi = 0; sgi < nalloc; ++sgi) {
    seg[sgi].G = (double *)calloc((size_t)(p * p), sizeof(double));
    seg[sgi].xtwz = (double *)calloc((size_t)p, sizeof(double));
  }
  double *Gm = malloc(sizeof(double) * (size_t)(p * p)), *xtwz = malloc(sizeof(double) * (size_t)p);
  double *coefs = calloc((size_t)p, sizeof(double)), *diag_design = calloc((size_t)p, sizeof(double));
  double s[ORC_NS];
  const double fac = family_dev_factor(o->family);
  int rc = ORC_OK;

  stream_pass(&g, row0, n, o->family, o->link, SP_YSUM, NULL, 0.0, o->nthreads, seg, nseg);
  seg_total(seg, p, 0, NULL, NULL, s, nseg);
  const double ymean = s[ORC_S_DEV] / (double)n; /* GLM.scala:263 / 423 */
  const int init = o->npart > 1 ? ORC_MODE_INIT_MULTI : ORC_MODE_INIT_SINGLE;
  stream_pass(&g, row0, n, o->family, o->link, init, NULL, ymean, o->nthreads, seg, nseg);
  seg_total(seg, p, 1, Gm, xtwz, s, nseg);
  double dev = fac * s[ORC_S_DEV], null_dev = dev, dev_old, deltad = 1.0;
  int iter = 0;
  if (out->dev_trace && out->max_trace > 0) out->dev_trace[0] = dev;
  while (fabs(deltad) > o->tol) { /* GLM.scala:281 / 452 */
    if (o->max_iter > 0 && iter >= o->max_iter) break;
    rc = wls_solve(Gm, xtwz, p, coefs, diag_design); /* wlsSingle (utils.scala:98-107) */
    if (rc) goto done;
    stream_pass(&g, row0, n, o->family, o->link, ORC_MODE_IRLS, coefs, ymean, o->nthreads, seg, nseg);
    seg_total(seg, p, 1, Gm, xtwz, s, nseg);
    dev_old = dev;
    dev = fac * s[ORC_S_DEV];
    deltad = dev - dev_old;
    iter = iter + 1;
    if (out->dev_trace && iter < out->max_trace) out->dev_trace[iter] = dev;
    if (o->verbose) { printf("%d\t%.17g\n", iter, deltad); fflush(stdout); }
  }
  if (s[ORC_S_BAD] > 0) { rc = ORC_EINVAL; goto done; }
  {
    double ll = s[ORC_S_LL];
    if (o->family == ORC_GAUSSIAN) {
      ll = -((double)n / 2.0) * (log(2.0 * M_PI * dev / (double)n) + 1.0) + 0.5 * s[ORC_S_LL];
    } else if (o->family == ORC_GAMMA) {
      double sw = s[ORC_S_SUMW], disp = dev / sw, a = 1.0 / disp;
      ll = (a - 1.0) * s[ORC_S_LL] - s[ORC_S_AUX0] / disp - (lgamma(a) + a * log(disp)) * sw - a * s[ORC_S_AUX1];
    }
    memcpy(out->coefs, coefs, sizeof(double) * (size_t)p);
    memcpy(out->stderr_, diag_design, sizeof(double) * (size_t)p);
    out->deviance = dev;
    out->null_deviance = null_dev;
    out->pearson = s[ORC_S_PEARSON];
    out->loglik = ll;
    out->iter = iter;
    out->nrow = (double)n;
    out->npart = o->npart > 0 ? o->npart : 1;
  }
done:
  for (int sgi = 0; sgi < nalloc; ++sgi) { free(seg[sgi].G); free(seg[sgi].xtwz); }
  free(seg); free(Gm); free(xtwz); free(coefs); free(diag_design); free(g.bs);
  return rc;
}
