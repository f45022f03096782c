// solve.hpp -- host p x p solves (Cholesky with LU fallback).
#pragma once
#include <cstdint>
#include <vector>

namespace sglm {

int chol_factor(double* A, int64_t p);  // 0 ok, else 1-based failing column
void chol_solve(const double* L, int64_t p, const double* b, double* x);
void chol_inv_diag(const double* L, int64_t p, double* diag);
void chol_inverse(const double* L, int64_t p, double* Ainv);
int lu_inverse(double* A, int64_t p);  // 0 ok, 1 exactly singular
// min_j L_jj^2 / A_jj of a Cholesky factor L of A: the part of column j's weighted norm that
// the previous columns do not explain (1 - R_j^2), a scale-free collinearity measure; its
// inverse bounds cond(A) from below.
double chol_pivot_ratio(const double* L, const double* A, int64_t p);
// Below this ratio (cond(X'WX) >~ 1e6) Cholesky and the reference's LU inverse part by more
// than cond * eps ~ 1e-10 relative, so the solve switches to Breeze inv()'s algorithm.
constexpr double LU_SWITCH_RATIO = 1e-6;

// Keeps the factorisation of the last solve so that the standard errors of the
// returned fit come from the same X'WX as its coefficients (utils.scala:103-105).
class Solver {
 public:
  explicit Solver(int64_t p) : p_(p) {}
  int solve(const double* A, const double* b, double* x);  // 0 ok, 1 singular
  void inv_diag(double* d) const;
  void inverse(double* Ainv) const;
  bool has_factor() const { return kind_ != 0; }
  bool used_lu() const { return kind_ == 2; }

 private:
  int64_t p_;
  int kind_ = 0;  // 0 none, 1 Cholesky factor, 2 explicit LU inverse
  std::vector<double> fac_;
};

}  // namespace sglm
