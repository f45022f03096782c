/*
 * sglm_oracle.h -- CPU restatement of cafreeman/sparkGLM's lm()/glm() fitting path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline.  The product path (sparkglm_amd/, libsglm_hip.so) never links or calls it.
 *
 * Parity status: PARTIALLY PINNED.  The reference (Scala 2.10 / Spark 1.4) cannot be
 * built or run in this image (no JVM).  The reference holds ONE
 * numeric known answer for this path -- the iris LM R-squared string asserted at
 * R/pkg/tests/testthat/test_LM.R:44 -- and this restatement reproduces it
 * (tests/test_oracle.py).  Every GLM number is otherwise unpinned by the reference;
 * the restatement is cross-checked against independent numpy/scipy/sklearn fits.
 *
 * Enumerations are shared with include/sglm.h (same integer values).
 */
#ifndef SGLM_ORACLE_H
#define SGLM_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_BINOMIAL = 0, ORC_GAUSSIAN = 1, ORC_POISSON = 2, ORC_GAMMA = 3 };
enum { ORC_LOGIT = 0, ORC_PROBIT = 1, ORC_CLOGLOG = 2, ORC_IDENTITY = 3, ORC_LOG = 4, ORC_INVERSE = 5 };
enum { ORC_OK = 0, ORC_EINVAL = 1, ORC_ESINGULAR = 2 };

typedef struct {
  int family;      /* ORC_BINOMIAL ... */
  int link;        /* ORC_LOGIT ... */
  double tol;      /* absolute |delta deviance| tolerance, GLM.scala:281 */
  int max_iter;    /* 0 = unbounded (the reference has no guard) */
  int verbose;     /* GLM.scala:304 */
  int npart;       /* 1 -> fitSingleBinomial semantics; G>1 -> fitMultipleBinomial over G row partitions */
  int nthreads;    /* threads for the partitioned Gram (Spark local[N] analogue) */
  int plain_sums;  /* orc_fit_glm_synth only: 1 = the reference's summation order for the scalars --
                      per partition (npart contiguous slices) a plain running sum over its rows, as
                      the ones-vector dgemm of createBinomialDeviance (GLM.scala:168) computes it in
                      reference BLAS, then the partition totals summed plainly in partition order
                      (GLM.scala:404-407); 0 = compensated (Neumaier) sums (the default) */
} orc_opts;

typedef struct {
  double *coefs;       /* [p] caller-allocated */
  double *stderr_;     /* [p] caller-allocated */
  double deviance, null_deviance, pearson, loglik;
  int iter;
  double nrow;
  int npart;
  double *dev_trace;   /* optional [max_trace]: deviance after each iteration (index 0 = null deviance) */
  int max_trace;
} orc_preglm;

/* Full GLM fit (GLM.scala:254-315 / 410-468). X column-major n x p with leading dim ldx. */
int orc_fit_glm(const double *X, int64_t n, int64_t p, int64_t ldx,
                const double *y, const double *m, const double *offset, const double *prior,
                const orc_opts *opts, orc_preglm *out);

/* LM.fit (LM.scala:241-274): fills coefs[p], xtxi[p*p] (col-major), stderr[p] and scalars. */
int orc_fit_lm(const double *X, int64_t n, int64_t p, int64_t ldx, const double *y, int npart,
               int nthreads, double *coefs, double *xtxi, double *stderr_, double *sse,
               double *r2, double *fstat, double *sigma);

/* Pass modes (same values as the engine's sglm_backend.pass modes). */
enum { ORC_MODE_IRLS = 0, ORC_MODE_INIT_SINGLE = 1, ORC_MODE_INIT_MULTI = 2, ORC_MODE_LM_GRAM = 3, ORC_MODE_LM_RESID = 4 };

/* One shard's contribution to one IRLS pass, in the engine's packed wire format:
 *   packed[0 .. p(p+1)/2)     lower-triangular X'WX, row-major (i >= j): index i*(i+1)/2 + j
 *   packed[tri .. tri+p)      X'Wz
 *   packed[tri+p .. +8)       scalars (see ORC_S_* below)
 * Modes: IRLS at beta; INIT_SINGLE (mu = mu0, fitSingleBinomial) / INIT_MULTI (mu =
 * unlink(link(mu0)), fitMultipleBinomial) constant-eta passes (GLM.scala:263-272);
 * LM_GRAM (X'X, X'y, sum y, rows); LM_RESID (SSE, SSR, SST at beta around ybar). */
enum { ORC_S_DEV = 0, ORC_S_PEARSON, ORC_S_LL, ORC_S_BAD, ORC_S_AUX0, ORC_S_AUX1, ORC_S_AUX2, ORC_S_SUMW, ORC_NS };
int orc_shard_partials(const double *X, int64_t n, int64_t p, int64_t ldx,
                       const double *y, const double *m, const double *offset, const double *prior,
                       int family, int link, int mode, const double *beta, double mu0, double ybar,
                       double *packed);

/* Streaming fit of the seeded synthetic design (sparkglm_amd/synth.py generator, kinds 0-3,
 * rows [row0, row0+n)), regenerated chunk by chunk on every IRLS iteration: full-scale
 * parity without holding X in host RAM.  npart > 1 selects the
 * fitMultipleBinomial first step; m = 1.  Same outputs as orc_fit_glm. */
int orc_fit_glm_synth(int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed, const orc_opts *opts,
                      orc_preglm *out);
/* One pass of that streaming fit at beta (mode ORC_MODE_IRLS) or at mu0 (init modes): G [p*p]
 * col-major symmetric X'WX, xtwz [p], s [8] scalars, summed as orc_fit_glm_synth sums them. */
int orc_pass_synth(int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed, int family, int link, int mode,
                   const double *beta, double mu0, int nthreads, double *G, double *xtwz, double *s);
/* The generator itself (X column-major with ld = n; offset / prior only for kind 2, may be NULL). */
int orc_synth_rows(int kind, int64_t row0, int64_t n, int64_t p, uint64_t seed, double *X, double *y,
                   double *offset, double *prior);

/* Breeze inv() semantics: LU with partial pivoting (dgetrf) + inverse (dgetri). In place, col-major. */
int orc_lu_inverse(double *A, int64_t p);

/* Scalar building blocks exposed for unit tests. */
double orc_norm_cdf(double x);
double orc_norm_icdf(double q);
double orc_erfinv(double x);

#ifdef __cplusplus
}
#endif
#endif
