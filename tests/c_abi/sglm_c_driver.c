/*
 * sglm_c_driver.c -- the C-ABI boundary driven from plain C (C99, no C++ and no Python between
 * the caller and include/sglm.h): what the JNI binding of INTEGRATION.md does, compiled with gcc.
 * "the C-ABI is the tested boundary, exercised by a C++ test driver and Python ctypes
 * tests".  tests/test_c_driver.py builds it (tests/c_abi/Makefile) and checks its output against the
 * oracle.
 *
 *   sglm_c_driver cpu DATA   LM.fit over caller-computed partials (sglm_fit_lm_external), two
 *                            partitions on two threads joined by the in-process communicator
 *                            (sglm_local_comm_*), the SummaryLM text, and the requires / device
 *                            errors a JVM caller maps to exceptions -- no GPU needed
 *   sglm_c_driver gpu DATA   sglm_create(devs, 1), set_data, fit_glm (binomial / logit), fit_lm,
 *                            predict_new, the GLM summary text, destroy -- on device 0
 *
 * DATA: int64 n, int64 p, then X (n x p, column-major doubles), y (n doubles) for the GLM and yl
 * (n doubles) for the LM.  Output: one "key v1 v2 ..." line per quantity (%.17g), the summary text
 * between "summary_begin" / "summary_end" lines, "ok" last.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sglm.h"

static int64_t n_, p_;
static double *X_, *y_, *yl_;

static void die(const char *what, int st) {
  fprintf(stderr, "%s failed: status %d: %s\n", what, st, sglm_last_error());
  exit(2);
}

static int load(const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) return -1;
  if (fread(&n_, sizeof n_, 1, f) != 1 || fread(&p_, sizeof p_, 1, f) != 1) return -1;
  X_ = malloc(sizeof(double) * (size_t)(n_ * p_));
  y_ = malloc(sizeof(double) * (size_t)n_);
  yl_ = malloc(sizeof(double) * (size_t)n_);
  if (fread(X_, sizeof(double), (size_t)(n_ * p_), f) != (size_t)(n_ * p_)) return -1;
  if (fread(y_, sizeof(double), (size_t)n_, f) != (size_t)n_) return -1;
  if (fread(yl_, sizeof(double), (size_t)n_, f) != (size_t)n_) return -1;
  fclose(f);
  return 0;
}

static void print_vec(const char *key, const double *v, int64_t k) {
  printf("%s", key);
  for (int64_t i = 0; i < k; ++i) printf(" %.17g", v[i]);
  printf("\n");
}

/* ---- the external LM backend: one row partition [lo, hi) of the data, LM.scala:142-188 ---- */
typedef struct {
  int64_t lo, hi;
} shard;

static int lm_local_sums(void *ctx, double *out2) {
  const shard *s = ctx;
  double sy = 0.0;
  for (int64_t i = s->lo; i < s->hi; ++i) sy += yl_[i];
  out2[0] = sy;
  out2[1] = (double)(s->hi - s->lo);
  return 0;
}

/* packed: lower-triangular X'X row-major (i >= j at i(i+1)/2 + j) | X'y [p] | 8 scalars
 * mode 3 (LM Gram): scalars[0] = sum y, scalars[7] = rows; mode 4 (residuals at beta, ybar):
 * scalars[0] = SSE, [1] = sum (X beta - ybar)^2, [2] = sum (y - ybar)^2, [7] = rows */
static int lm_pass(void *ctx, int mode, const double *beta, double mu0, double ybar, double *packed) {
  (void)mu0;
  const shard *s = ctx;
  const int64_t p = p_, tri = p * (p + 1) / 2;
  memset(packed, 0, sizeof(double) * (size_t)(tri + p + 8));
  double *sc = packed + tri + p;
  for (int64_t r = s->lo; r < s->hi; ++r) {
    const double y = yl_[r];
    if (mode == 3) {
      for (int64_t i = 0; i < p; ++i) {
        const double xi = X_[r + i * n_];
        for (int64_t j = 0; j <= i; ++j) packed[i * (i + 1) / 2 + j] += xi * X_[r + j * n_];
        packed[tri + i] += xi * y;
      }
      sc[0] += y;
    } else if (mode == 4) {
      double eta = 0.0;
      for (int64_t j = 0; j < p; ++j) eta += X_[r + j * n_] * beta[j];
      const double e = y - eta, t = eta - ybar, b = y - ybar;
      sc[0] += e * e;
      sc[1] += t * t;
      sc[2] += b * b;
    } else {
      return 1; /* an LM backend answers only the LM modes */
    }
    sc[7] += 1.0;
  }
  return 0;
}

typedef struct {
  int rank;
  sglm_local_comm *comm;
  sglm_prelm pre;
  double coefs[64], se[64], xtxi[64 * 64];
  int st;
} lm_job;

static void *lm_thread(void *arg) {
  lm_job *j = arg;
  shard s = {j->rank == 0 ? 0 : n_ / 2, j->rank == 0 ? n_ / 2 : n_};
  sglm_backend be = {&s, p_, lm_local_sums, lm_pass};
  memset(&j->pre, 0, sizeof j->pre);
  j->pre.coefs = j->coefs;
  j->pre.std_err = j->se;
  j->pre.xtxi = j->xtxi;
  j->st = sglm_fit_lm_external(&be, sglm_local_allreduce, sglm_local_comm_rank(j->comm, j->rank), &j->pre);
  return NULL;
}

static int run_cpu(void) {
  if (p_ > 64) return 3;
  /* requires -> SGLM_EINVAL with the reference's message; no device -> SGLM_EHIP, no handle */
  sglm_engine *h = NULL;
  int devs[1] = {0};
  printf("create_null_devs %d\n", sglm_create(NULL, 1, &h));
  printf("create_zero_devs %d\n", sglm_create(devs, 0, &h));
  int ndev = -1;
  const int dc = sglm_device_count(&ndev);
  if (dc != 0 || ndev == 0) printf("create_no_device %d %d\n", sglm_create(devs, 1, &h), h == NULL);
  printf("abi %d\n", sglm_abi_version());

  sglm_local_comm *comm = NULL;
  int st = sglm_local_comm_create(2, &comm);
  if (st) die("sglm_local_comm_create", st);
  lm_job jobs[2];
  pthread_t th[2];
  for (int r = 0; r < 2; ++r) {
    jobs[r].rank = r;
    jobs[r].comm = comm;
    pthread_create(&th[r], NULL, lm_thread, &jobs[r]);
  }
  for (int r = 0; r < 2; ++r) pthread_join(th[r], NULL);
  sglm_local_comm_destroy(comm);
  for (int r = 0; r < 2; ++r)
    if (jobs[r].st) die("sglm_fit_lm_external", jobs[r].st);
  printf("ranks_bitwise %d\n", memcmp(jobs[0].coefs, jobs[1].coefs, sizeof(double) * (size_t)p_) == 0 &&
                                   memcmp(jobs[0].se, jobs[1].se, sizeof(double) * (size_t)p_) == 0);
  const sglm_prelm *pre = &jobs[0].pre;
  print_vec("lm_coefs", pre->coefs, p_);
  print_vec("lm_stderr", pre->std_err, p_);
  const double sc[5] = {pre->sse, pre->r2, pre->fstat, pre->sigma, pre->nrow};
  print_vec("lm_stats", sc, 5);
  printf("lm_npart %d\n", pre->npart);

  char names[64][16];
  const char *xn[64];
  for (int64_t j = 0; j < p_; ++j) {
    snprintf(names[j], sizeof names[j], "x%d", (int)j);
    xn[j] = names[j];
  }
  const int64_t need = sglm_lm_summary(pre, p_, xn, "y", NULL, 0);
  char *buf = malloc((size_t)need);
  sglm_lm_summary(pre, p_, xn, "y", buf, need);
  printf("summary_begin\n%ssummary_end\n", buf);
  free(buf);
  printf("ok\n");
  return 0;
}

static int run_gpu(void) {
  sglm_engine *h = NULL;
  int devs[1] = {0};
  int st = sglm_create(devs, 1, &h);
  if (st) die("sglm_create", st);
  /* a require that fails before any device work */
  printf("set_data_bad_n %d\n", sglm_set_data(h, X_, 0, p_, n_, y_, NULL, NULL, NULL));
  st = sglm_set_data(h, X_, n_, p_, n_, y_, NULL, NULL, NULL);
  if (st) die("sglm_set_data", st);

  double coefs[64], se[64], trace[64];
  sglm_glm_opts o = {SGLM_BINOMIAL, SGLM_LOGIT, 1e-6, 0, 0, SGLM_INIT_SINGLE, 0};
  sglm_preglm g;
  memset(&g, 0, sizeof g);
  g.coefs = coefs;
  g.std_err = se;
  g.dev_trace = trace;
  g.max_trace = 64;
  st = sglm_fit_glm(h, &o, &g);
  if (st) die("sglm_fit_glm", st);
  print_vec("glm_coefs", coefs, p_);
  print_vec("glm_stderr", se, p_);
  const double gs[5] = {g.deviance, g.null_deviance, g.pearson, g.loglik, g.nrow};
  print_vec("glm_stats", gs, 5);
  printf("glm_iter %d\n", g.iter);

  double *eta = malloc(sizeof(double) * (size_t)n_);
  st = sglm_predict_new(h, X_, n_, p_, n_, coefs, NULL, NULL, SGLM_BINOMIAL, SGLM_LOGIT, SGLM_PREDICT_RESPONSE, eta);
  if (st) die("sglm_predict_new", st);
  print_vec("mu_head", eta, n_ < 5 ? n_ : 5);
  free(eta);

  char names[64][16];
  const char *xn[64];
  for (int64_t j = 0; j < p_; ++j) {
    snprintf(names[j], sizeof names[j], "x%d", (int)j);
    xn[j] = names[j];
  }
  const int64_t need = sglm_glm_summary(&g, p_, xn, "y", "binomial", "logit", NULL, 0);
  char *text = malloc((size_t)need);
  sglm_glm_summary(&g, p_, xn, "y", "binomial", "logit", text, need);
  printf("summary_begin\n%ssummary_end\n", text);
  free(text);

  /* LM on the same design: the gaussian response */
  st = sglm_set_data(h, X_, n_, p_, n_, yl_, NULL, NULL, NULL);
  if (st) die("sglm_set_data (lm)", st);
  double lc[64], lse[64];
  sglm_prelm l;
  memset(&l, 0, sizeof l);
  l.coefs = lc;
  l.std_err = lse;
  st = sglm_fit_lm(h, &l);
  if (st) die("sglm_fit_lm", st);
  print_vec("lm_coefs", lc, p_);
  print_vec("lm_stderr", lse, p_);
  const double ls[5] = {l.sse, l.r2, l.fstat, l.sigma, l.nrow};
  print_vec("lm_stats", ls, 5);

  sglm_stats stt;
  st = sglm_get_stats(h, &stt);
  if (st) die("sglm_get_stats", st);
  printf("kernel %s\n", stt.pass_kernel_name);
  sglm_destroy(h);
  printf("ok\n");
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 3 || load(argv[2]) != 0 || p_ < 1 || p_ > 64) {
    fprintf(stderr, "usage: sglm_c_driver cpu|gpu DATA (1 <= p <= 64)\n");
    return 1;
  }
  return strcmp(argv[1], "gpu") == 0 ? run_gpu() : run_cpu();
}
