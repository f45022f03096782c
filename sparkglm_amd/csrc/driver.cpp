// driver.cpp -- the IRLS (Fisher scoring) and least-squares drivers.
//
// glm_drive restates the loop of GLM.fitSingleBinomial (GLM.scala:254-315) and
// GLM.fitMultipleBinomial (GLM.scala:410-468) over any Backend:
//   mu0 = mean(y); eta0 = link(mu0) with the offset ignored; dev0 = nullDeviance
//   while |dev_k - dev_{k-1}| > tol (absolute; deltad starts at 1.0):
//       beta = solve(X'WX, X'Wz)          (wlsSingle / wlsMultiple)
//       eta = X beta + offset; mu = unlink(eta); dev = deviance(mu)   (one fused pass)
//   stdErr = sqrt(diag(inv(X'WX))) of the last solve; pearson / loglik at the final mu.
// Each backend pass returns the NEXT iteration's X'WX together with the current deviance,
// so one pass over X serves both halves of a reference iteration.
#include "driver.hpp"

#include <chrono>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "solve.hpp"

extern "C" int64_t sglm_java_double_string(double x, char* buf, int64_t buflen);

namespace sglm {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* get_error() { return g_err.c_str(); }

int family_link_valid(int family, int link) {
  switch (family) {
    case FAM_BINOMIAL: return link == LNK_LOGIT || link == LNK_PROBIT || link == LNK_CLOGLOG;
    case FAM_GAUSSIAN: return link == LNK_IDENTITY;
    case FAM_POISSON: return link == LNK_LOG;
    case FAM_GAMMA: return link == LNK_INVERSE;
    default: return 0;
  }
}

double family_dev_factor(int family) { return family == FAM_GAUSSIAN ? 1.0 : 2.0; }

void unpack_gram(const double* packed, int64_t p, double* gram, double* xtwz) {
  for (int64_t i = 0; i < p; ++i)
    for (int64_t j = 0; j <= i; ++j) {
      const double v = packed[i * (i + 1) / 2 + j];
      gram[i + j * p] = v;
      gram[j + i * p] = v;
    }
  std::memcpy(xtwz, packed + tri_count(p), sizeof(double) * (size_t)p);
}

struct HostSolver::Impl {
  Solver s;
  explicit Impl(int64_t p) : s(p) {}
};
HostSolver::HostSolver(int64_t p) : p_(p), gram_((size_t)(p * p)), rhs_((size_t)p), impl_(new Impl(p)) {}
HostSolver::~HostSolver() = default;
int HostSolver::solve(const double* packed, double* x) {
  unpack_gram(packed, p_, gram_.data(), rhs_.data());
  return impl_->s.solve(gram_.data(), rhs_.data(), x) ? SGLM_ESINGULAR : SGLM_OK;
}
int HostSolver::inv_diag(double* d) {
  impl_->s.inv_diag(d);
  return SGLM_OK;
}
int HostSolver::inverse(double* Ainv) {
  impl_->s.inverse(Ainv);
  return SGLM_OK;
}
int HostSolver::path() const {
  return !impl_->s.has_factor() ? -1 : impl_->s.used_lu() ? SGLM_SOLVE_HOST_LU : SGLM_SOLVE_HOST_CHOL;
}

static double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// Loglik from the final-statistics scalars (families without per-row closed forms).
static double family_loglik(int family, const double* s, double dev, double nrow) {
  if (family == FAM_GAUSSIAN) {
    // R gaussian()$aic with sigma^2 = dev/n: -(n/2)(log(2 pi dev/n) + 1) + 0.5 sum(log w)
    return -(nrow / 2.0) * (std::log(2.0 * M_PI * dev / nrow) + 1.0) + 0.5 * s[S_LL];
  }
  if (family == FAM_GAMMA) {
    // R Gamma()$aic: disp = dev / sum(w); sum w * dgamma(y, 1/disp, scale = mu*disp, log)
    const double sw = s[S_SUMW], disp = dev / sw, a = 1.0 / disp;
    return (a - 1.0) * s[S_LL] - s[S_AUX0] / disp - (std::lgamma(a) + a * std::log(disp)) * sw - a * s[S_AUX1];
  }
  return s[S_LL];
}

int glm_drive(Backend& be, const sglm_glm_opts& o, sglm_preglm* out) {
  if (!family_link_valid(o.family, o.link)) {
    set_error("requirement failed: unsupported family/link combination");
    return SGLM_EINVAL;
  }
  const int64_t p = be.ncols();
  const size_t pk = (size_t)packed_len(p);
  std::vector<double> packed(pk), beta((size_t)p, 0.0), s(NS);
  std::unique_ptr<SolverIface> solver = be.make_solver(p);
  double sums[2];
  int rc = be.global_sums(sums);
  if (rc) return rc;
  const double nrow = sums[1];
  if (!(nrow > 0)) {
    set_error("requirement failed: The number of rows must be strictly greater than 0");
    return SGLM_EINVAL;
  }
  const double ymean = sums[0] / nrow;  // GLM.scala:263 / 423
  const double fac = family_dev_factor(o.family);
  const int init_mode = (o.init_mode == SGLM_INIT_MULTIPLE) ? MODE_INIT_MULTI : MODE_INIT_SINGLE;

  rc = be.pass(init_mode, nullptr, ymean, 0.0, o.family, o.link, packed.data());
  if (rc) return rc;
  double dev = fac * packed[tri_count(p) + p + S_DEV];
  const double null_dev = dev;  // GLM.scala:272 / 444
  double deltad = 1.0, d_prev = 0.0;  // d_prev: |deltad| of the iteration before (speculation)
  int iter = 0;
  if (out->dev_trace && out->max_trace > 0) out->dev_trace[0] = dev;

  while (std::fabs(deltad) > o.tol) {  // GLM.scala:281 / 452
    if (o.max_iter > 0 && iter >= o.max_iter) break;
    const double t0 = now_ms();
    const int srv = solver->solve(packed.data(), beta.data());
    be.solve_ms += now_ms() - t0;
    be.solve_path = solver->path();
    if (srv) {
      if (srv == SGLM_ESINGULAR) set_error("breeze.linalg.MatrixSingularException: X'WX is singular");
      return srv;
    }
    // Speculative last pass: IRLS converges quadratically, so from the last two changes the next
    // one is predicted as d_k^3 / d_{k-1}^2; when that is below tol / 10 the pass at beta is run
    // without its Gram (which only the next solve would use).  If the deviance then shows no
    // convergence after all, the full pass at the same beta follows -- the scalars are bitwise
    // those of the full pass either way, so the fit is identical with or without speculation.
    bool spec = false;
    if (be.has_dev_pass() && iter >= 2 && d_prev > 0.0 && !(o.max_iter > 0 && iter + 1 >= o.max_iter)) {
      const double dk = std::fabs(deltad);
      spec = dk * dk * dk < 0.1 * o.tol * d_prev * d_prev;
    }
    if (spec) {
      rc = be.pass_dev(MODE_IRLS, beta.data(), ymean, 0.0, o.family, o.link, packed.data());
      if (rc) return rc;
      if (!(std::fabs(fac * packed[tri_count(p) + p + S_DEV] - dev) <= o.tol))
        spec = false;  // not the last iteration after all: the full pass at the same beta
    }
    if (!spec) {
      rc = be.pass(MODE_IRLS, beta.data(), ymean, 0.0, o.family, o.link, packed.data());
      if (rc) return rc;
    }
    const double dev_old = dev;
    d_prev = std::fabs(deltad);
    dev = fac * packed[tri_count(p) + p + S_DEV];
    deltad = dev - dev_old;
    iter = iter + 1;
    if (out->dev_trace && iter < out->max_trace) out->dev_trace[iter] = dev;
    if (o.verbose) {  // println(iter.toString + "\t" + deltad.toString)  (GLM.scala:304)
      char buf[64];
      sglm_java_double_string(deltad, buf, sizeof buf);
      std::printf("%d\t%s\n", iter, buf);
      std::fflush(stdout);
    }
  }

  if (iter > 0 && be.pass_has_stats()) {  // the last pass computed them at the final mu
    std::memcpy(s.data(), packed.data() + tri_count(p) + p, sizeof(double) * NS);
  } else {
    rc = be.stats(iter > 0 ? MODE_IRLS : init_mode, beta.data(), ymean, 0.0, o.family, o.link, s.data());
    if (rc) return rc;
  }
  if (s[S_BAD] > 0) {
    set_error("requirement failed: Binomial(m.toInt, mu).logProbabilityOf(y.toInt) needs 0 <= y <= m, m >= 1");
    return SGLM_EINVAL;
  }
  std::vector<double> d((size_t)p, 0.0);
  if (iter > 0) {
    rc = solver->inv_diag(d.data());
    if (rc) return rc;
  }
  for (int64_t i = 0; i < p; ++i) {
    out->coefs[i] = beta[i];
    out->std_err[i] = std::sqrt(d[i]);  // GLM.scala:307 / 464 (utils.scala:105)
  }
  out->deviance = dev;
  out->null_deviance = null_dev;
  out->pearson = s[S_PEARSON];
  out->loglik = family_loglik(o.family, s.data(), dev, nrow);
  out->iter = iter;
  out->nrow = nrow;
  out->npart = o.npart > 0 ? o.npart : be.npart();
  return SGLM_OK;
}

int irls_iterate(Backend& be, const sglm_glm_opts& o, double* beta, int iters, double* last_dev) {
  if (!family_link_valid(o.family, o.link)) {
    set_error("requirement failed: unsupported family/link combination");
    return SGLM_EINVAL;
  }
  const int64_t p = be.ncols();
  std::vector<double> packed((size_t)packed_len(p));
  std::unique_ptr<SolverIface> solver = be.make_solver(p);
  for (int it = 0; it < iters; ++it) {
    int rc = be.pass(MODE_IRLS, beta, 0.0, 0.0, o.family, o.link, packed.data());
    if (rc) return rc;
    if (last_dev) *last_dev = family_dev_factor(o.family) * packed[tri_count(p) + p + S_DEV];
    const double t0 = now_ms();
    const int srv = solver->solve(packed.data(), beta);
    be.solve_ms += now_ms() - t0;
    be.solve_path = solver->path();
    if (srv) {
      if (srv == SGLM_ESINGULAR) set_error("breeze.linalg.MatrixSingularException: X'WX is singular");
      return srv;
    }
  }
  return SGLM_OK;
}

// LM.fit (LM.scala:241-274) over fitMultiple's components (LM.scala:217-237).
int lm_drive(Backend& be, sglm_prelm* out) {
  const int64_t p = be.ncols();
  std::vector<double> packed((size_t)packed_len(p)), s(NS), dev_coefs((size_t)p);
  bool dev = false;  // Gram pass, device solve and residual pass in one round trip (Backend::lm_device)
  int rc = be.lm_device(packed.data(), dev_coefs.data(), s.data(), dev);
  if (rc) return rc;
  if (!dev) rc = be.pass(MODE_LM_GRAM, nullptr, 0.0, 0.0, FAM_GAUSSIAN, LNK_IDENTITY, packed.data());
  if (rc) return rc;
  const double ysum = packed[tri_count(p) + p + S_DEV], nrow = packed[tri_count(p) + p + S_SUMW];
  std::unique_ptr<SolverIface> solver = be.make_solver(p);
  std::vector<double> coefs((size_t)p), xtxi((size_t)(p * p));
  const double t0 = now_ms();
  // coefs = inv(X'X) * X'y (LM.scala:225-227); the Cholesky solve is the same product.
  const int srv = solver->solve(packed.data(), coefs.data());
  if (srv) {
    if (srv == SGLM_ESINGULAR) set_error("breeze.linalg.MatrixSingularException: X'X is singular");
    return srv;
  }
  rc = solver->inverse(xtxi.data());
  if (rc) return rc;
  be.solve_ms += now_ms() - t0;
  be.solve_path = solver->path();
  const double ymean = ysum / nrow;  // LM.scala:167-168
  // the device's residual statistics stand only if its solve was this one, bit for bit; a device
  // Cholesky that failed a pivot returns NaN coefficients (its statistics are never used)
  const bool dev_failed = dev && std::any_of(dev_coefs.begin(), dev_coefs.end(), [](double v) { return std::isnan(v); });
  // ... and only if the sums they were formed from did not cancel too far (S_BAD: lm_chol_kernel's
  // LM_ONEPASS_MAX_RATIO guard) -- otherwise the residual pass, LM.scala:160-188's own form
  if (!dev || dev_failed || s[S_BAD] != 0.0 ||
      std::memcmp(dev_coefs.data(), coefs.data(), sizeof(double) * (size_t)p) != 0) {
    rc = be.stats(MODE_LM_RESID, coefs.data(), 0.0, ymean, FAM_GAUSSIAN, LNK_IDENTITY, s.data());
    if (rc) return rc;
    if (dev) be.lm_device_reruns += 1;
  }
  const double sse = s[S_DEV], top = s[S_PEARSON], bot = s[S_LL];
  const double r2 = top / bot;                                                      // LM.scala:185
  const double fstat = ((bot - sse) / ((double)p - 1.0)) / (sse / (nrow - (double)p));  // LM.scala:186
  const double sig2 = sse / (nrow - (double)p);                                      // LM.scala:260
  for (int64_t i = 0; i < p; ++i) {
    out->coefs[i] = coefs[i];
    out->std_err[i] = std::sqrt(sig2 * xtxi[i + i * p]);  // LM.scala:262-263
  }
  if (out->xtxi) std::memcpy(out->xtxi, xtxi.data(), sizeof(double) * (size_t)(p * p));
  out->sse = sse;
  out->r2 = r2;
  out->fstat = fstat;
  out->sigma = std::sqrt(sig2);
  out->nrow = nrow;
  out->npart = be.npart();
  return SGLM_OK;
}

}  // namespace sglm
