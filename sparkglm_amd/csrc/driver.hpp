// driver.hpp -- backend-agnostic IRLS / least-squares drivers (host side).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/sglm.h"
#include "common.hpp"

namespace sglm {

void set_error(const std::string& msg);
const char* get_error();

// The p x p solve of one iteration.  solve() takes the all-reduced packed pass output and
// keeps what it needs for inv_diag() / inverse() of the same matrix (the standard errors
// come from the last solve, utils.scala:103-105).  Returns SGLM_OK, SGLM_ESINGULAR, or
// another status with the error message set.
class SolverIface {
 public:
  virtual ~SolverIface() = default;
  virtual int solve(const double* packed, double* x) = 0;
  virtual int inv_diag(double* d) = 0;
  virtual int inverse(double* Ainv) = 0;
  // enum sglm_solve_path of the last solve (-1 before any)
  virtual int path() const = 0;
};

// Host Cholesky with the LU fallback (solve.cpp).
class HostSolver : public SolverIface {
 public:
  explicit HostSolver(int64_t p);
  ~HostSolver() override;
  int solve(const double* packed, double* x) override;
  int inv_diag(double* d) override;
  int inverse(double* Ainv) override;
  int path() const override;

 private:
  int64_t p_;
  std::vector<double> gram_, rhs_;
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

// A producer of all-reduced pass results.  The HIP engine implements it over its
// resident shard + communicator; sglm_fit_*_external adapts caller callbacks.
class Backend {
 public:
  virtual ~Backend() = default;
  virtual int64_t ncols() const = 0;
  virtual int npart() const = 0;  // number of shards (ranks) joined by the communicator
  // {sum y, rows} over all shards
  virtual int global_sums(double* out2) = 0;
  // One pass in the packed wire format (lower tri X'WX | X'Wz | NS scalars), all-reduced.
  virtual int pass(int mode, const double* beta, double mu0, double ybar, int family, int link, double* packed) = 0;
  // Final statistics (pearson, loglik ingredients, ...) at the state of the last pass
  // (MODE_IRLS / init modes) or at beta (MODE_LM_RESID), all-reduced, NS scalars.
  virtual int stats(int mode, const double* beta, double mu0, double ybar, int family, int link, double* s) = 0;
  // True when the last MODE_IRLS pass also delivered the final statistics (pearson, loglik
  // ingredients, bad) in its packed scalars, so glm_drive needs no stats() pass.
  virtual bool pass_has_stats() const { return false; }
  // Deviance-only pass: the scalars of pass() at beta (bitwise), no Gram.  glm_drive runs it
  // for an iteration it predicts to be the last (the Gram of that pass would go unused).
  virtual bool has_dev_pass() const { return false; }
  virtual int pass_dev(int mode, const double* beta, double mu0, double ybar, int family, int link, double* packed) {
    return pass(mode, beta, mu0, ybar, family, link, packed);
  }
  // LM.fit in one device round trip (lm_drive): the LM Gram pass, a device Cholesky solve in the
  // host solver's exact operation order, and the residual pass at those coefficients, with one
  // synchronisation.  Fills packed (the all-reduced Gram pass), dev_coefs and s (the residual
  // statistics at dev_coefs) and sets done; done = false: not available here (lm_drive then takes
  // the host round trips).  lm_drive keeps its host solve as the arbiter: when that solve does not
  // reproduce dev_coefs bitwise (the LU fallback of an ill-conditioned X'X) it reruns the residual
  // pass at its own coefficients.
  virtual int lm_device(double* packed, double* dev_coefs, double* s, bool& done) {
    (void)packed;
    (void)dev_coefs;
    (void)s;
    done = false;
    return SGLM_OK;
  }
  // The solver for this backend's systems (default: host).
  virtual std::unique_ptr<SolverIface> make_solver(int64_t p) { return std::make_unique<HostSolver>(p); }
  // host-side timers (ms) for sglm_stats
  double solve_ms = 0.0;
  int64_t lm_device_reruns = 0;  // device LM fits whose coefficients were not the host solve's (residual pass rerun)
  int solve_path = -1;  // enum sglm_solve_path of the last solve
};

int glm_drive(Backend& be, const sglm_glm_opts& o, sglm_preglm* out);
int lm_drive(Backend& be, sglm_prelm* out);
// Bench / test helper: `iters` IRLS iterations (pass at beta, then solve) from beta.
int irls_iterate(Backend& be, const sglm_glm_opts& o, double* beta, int iters, double* last_dev);

void unpack_gram(const double* packed, int64_t p, double* gram, double* xtwz);
int family_link_valid(int family, int link);
double family_dev_factor(int family);

}  // namespace sglm
