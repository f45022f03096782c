// solve.cpp -- host p x p solves for the IRLS / LM drivers.
//
// The reference inverts X'WX with Breeze inv() (LAPACK dgetrf + dgetri) and multiplies
// (utils.scala:103-105, 134-136; LM.scala:197-199, 225-227).  X'WX is symmetric positive
// definite whenever every working weight is positive, so the engine factors it with
// Cholesky (half the flops of LU, no pivot search) and keeps the factor of the last solve
// for the standard errors.  Two cases take the reference's own algorithm, LU with partial
// pivoting and the explicit inverse: a matrix Cholesky rejects (negative weights from the
// reference's unguarded formulas, or numerical indefiniteness), and an ill-conditioned one
// (chol_pivot_ratio < LU_SWITCH_RATIO, cond >~ 1e6), where the two algorithms' rounding
// parts by cond * eps -- past the 1e-9 parity bar at cond ~1e7 (tests/test_host_paths.py).
// An exactly singular matrix is reported like Breeze's MatrixSingularException.
#include "solve.hpp"

#include <cmath>
#include <cstring>
#include <vector>

namespace sglm {

// Left-looking (jki) Cholesky on a column-major full matrix; lower triangle out.  Four columns at a
// time: the panel's update by the columns before it streams each of those columns once for all four
// (the p = 256 solve of every configs[1] iteration: 0.86 -> 0.3 ms on one core), then the panel
// factors column by column.  Every element still subtracts its terms in k order, one rounding each,
// so the factor is bitwise the column-by-column one (the rows above the diagonal that the panel
// update also touches are never read and are zeroed at the end).
int chol_factor(double* A, int64_t p) {
  constexpr int64_t NB = 4;
  for (int64_t j0 = 0; j0 < p; j0 += NB) {
    const int64_t nb = p - j0 < NB ? p - j0 : NB;
    double* P = A + j0 * p;  // the panel's first column
    // the panel's update by the columns k < j0.  Dense panel (no zero multiplier): 8-row blocks of the
    // four columns stay in registers over the whole k loop; otherwise column by column with the
    // zero multipliers skipped, as the unblocked loop does
    bool dense = nb == NB;
    for (int64_t k = 0; k < j0 && dense; ++k)
      for (int64_t c = 0; c < NB; ++c) dense = dense && A[j0 + c + k * p] != 0.0;
    if (dense) {
      constexpr int64_t R = 8;
      int64_t i0 = j0;
      for (; i0 + R <= p; i0 += R) {
        double acc[NB][R];
        for (int64_t c = 0; c < NB; ++c)
          for (int64_t r = 0; r < R; ++r) acc[c][r] = P[c * p + i0 + r];
        for (int64_t k = 0; k < j0; ++k) {
          const double* Ak = A + k * p;
          const double* lk = A + k * p + j0;
          for (int64_t c = 0; c < NB; ++c) {
            const double l = lk[c];
            for (int64_t r = 0; r < R; ++r) acc[c][r] -= Ak[i0 + r] * l;
          }
        }
        for (int64_t c = 0; c < NB; ++c)
          for (int64_t r = 0; r < R; ++r) P[c * p + i0 + r] = acc[c][r];
      }
      for (int64_t k = 0; k < j0 && i0 < p; ++k) {  // the last rows
        const double* Ak = A + k * p;
        for (int64_t c = 0; c < NB; ++c) {
          const double l = A[j0 + c + k * p];
          for (int64_t i = i0; i < p; ++i) P[c * p + i] -= Ak[i] * l;
        }
      }
    } else {
      for (int64_t k = 0; k < j0; ++k) {
        const double* Ak = A + k * p;
        for (int64_t c = 0; c < nb; ++c) {
          const double l = A[j0 + c + k * p];
          if (l == 0.0) continue;
          double* Pc = P + c * p;
          for (int64_t i = j0; i < p; ++i) Pc[i] -= Ak[i] * l;
        }
      }
    }
    for (int64_t j = j0; j < j0 + nb; ++j) {
      double* Aj = A + j * p;
      for (int64_t k = j0; k < j; ++k) {
        const double ljk = A[j + k * p];
        if (ljk == 0.0) continue;
        const double* Ak = A + k * p;
        for (int64_t i = j; i < p; ++i) Aj[i] -= Ak[i] * ljk;
      }
      const double d = Aj[j];
      if (!(d > 0.0) || !std::isfinite(d)) return (int)(j + 1);
      const double s = std::sqrt(d);
      Aj[j] = s;
      const double inv = 1.0 / s;
      for (int64_t i = j + 1; i < p; ++i) Aj[i] *= inv;
    }
  }
  for (int64_t j = 1; j < p; ++j)
    for (int64_t i = 0; i < j; ++i) A[i + j * p] = 0.0;
  return 0;
}

void chol_solve(const double* L, int64_t p, const double* b, double* x) {
  std::vector<double> t(b, b + p);
  for (int64_t j = 0; j < p; ++j) {  // L t = b (column sweep)
    t[j] /= L[j + j * p];
    const double tj = t[j];
    for (int64_t i = j + 1; i < p; ++i) t[i] -= L[i + j * p] * tj;
  }
  for (int64_t i = p - 1; i >= 0; --i) {  // L' x = t (column sweep: x_i, then t_k -= L(i, k) x_i, k < i)
    t[i] /= L[i + i * p];
    const double xi = t[i];
    for (int64_t k = 0; k < i; ++k) t[k] -= L[i + k * p] * xi;
  }
  std::memcpy(x, t.data(), sizeof(double) * p);
}

// inv(L) in place-free form: returns M = inv(L) (lower), column-major.
static void tri_inverse(const double* L, int64_t p, std::vector<double>& M) {
  M.assign((size_t)(p * p), 0.0);
  for (int64_t j = 0; j < p; ++j) {
    double* Mj = M.data() + j * p;
    Mj[j] = 1.0 / L[j + j * p];
    for (int64_t i = j + 1; i < p; ++i) {
      // M[i][j] = -(sum_{k=j}^{i-1} L[i][k] M[k][j]) / L[i][i]
      double s = 0.0;
      for (int64_t k = j; k < i; ++k) s += L[i + k * p] * Mj[k];
      Mj[i] = -s / L[i + i * p];
    }
  }
}

void chol_inv_diag(const double* L, int64_t p, double* diag) {
  std::vector<double> M;
  tri_inverse(L, p, M);
  for (int64_t i = 0; i < p; ++i) {  // inv(A) = M' M  ->  diag_i = sum_k M[k][i]^2
    const double* Mi = M.data() + i * p;
    double s = 0.0;
    for (int64_t k = i; k < p; ++k) s += Mi[k] * Mi[k];
    diag[i] = s;
  }
}

void chol_inverse(const double* L, int64_t p, double* Ainv) {
  std::vector<double> M;
  tri_inverse(L, p, M);
  for (int64_t j = 0; j < p; ++j)
    for (int64_t i = j; i < p; ++i) {
      const double* Mi = M.data() + i * p;
      const double* Mj = M.data() + j * p;
      double s = 0.0;
      for (int64_t k = i; k < p; ++k) s += Mi[k] * Mj[k];
      Ainv[i + j * p] = s;
      Ainv[j + i * p] = s;
    }
}

int lu_inverse(double* A, int64_t p) {
  std::vector<int64_t> piv((size_t)p);
  for (int64_t k = 0; k < p; ++k) {
    int64_t ip = k;
    double amax = std::fabs(A[k + k * p]);
    for (int64_t i = k + 1; i < p; ++i)
      if (std::fabs(A[i + k * p]) > amax) { amax = std::fabs(A[i + k * p]); ip = i; }
    piv[k] = ip;
    if (A[ip + k * p] == 0.0) return 1;
    if (ip != k)
      for (int64_t j = 0; j < p; ++j) std::swap(A[k + j * p], A[ip + j * p]);
    const double inv = 1.0 / A[k + k * p];
    for (int64_t i = k + 1; i < p; ++i) A[i + k * p] *= inv;
    for (int64_t j = k + 1; j < p; ++j) {
      const double a = A[k + j * p];
      if (a != 0.0)
        for (int64_t i = k + 1; i < p; ++i) A[i + j * p] -= A[i + k * p] * a;
    }
  }
  for (int64_t j = 0; j < p; ++j) {  // inv(U)
    A[j + j * p] = 1.0 / A[j + j * p];
    const double ajj = -A[j + j * p];
    for (int64_t k = 0; k < j; ++k) {
      const double t = A[k + j * p];
      if (t != 0.0) {
        for (int64_t i = 0; i < k; ++i) A[i + j * p] += t * A[i + k * p];
        A[k + j * p] = t * A[k + k * p];
      }
    }
    for (int64_t i = 0; i < j; ++i) A[i + j * p] *= ajj;
  }
  std::vector<double> work((size_t)p);
  for (int64_t j = p - 1; j >= 0; --j) {  // inv(A) L = inv(U)
    for (int64_t i = j + 1; i < p; ++i) { work[i] = A[i + j * p]; A[i + j * p] = 0.0; }
    for (int64_t k = j + 1; k < p; ++k) {
      const double t = work[k];
      if (t != 0.0)
        for (int64_t i = 0; i < p; ++i) A[i + j * p] -= A[i + k * p] * t;
    }
  }
  for (int64_t j = p - 2; j >= 0; --j) {
    const int64_t jp = piv[j];
    if (jp != j)
      for (int64_t i = 0; i < p; ++i) std::swap(A[i + j * p], A[i + jp * p]);
  }
  return 0;
}

double chol_pivot_ratio(const double* L, const double* A, int64_t p) {
  double r = 1.0;
  for (int64_t j = 0; j < p; ++j) {
    const double l = L[j + j * p], a = A[j + j * p];
    if (a > 0.0) r = std::fmin(r, (l * l) / a);
  }
  return r;
}

int Solver::solve(const double* A, const double* b, double* x) {
  const size_t pp = (size_t)(p_ * p_);
  fac_.assign(A, A + pp);
  if (chol_factor(fac_.data(), p_) == 0 && chol_pivot_ratio(fac_.data(), A, p_) >= LU_SWITCH_RATIO) {
    kind_ = 1;
    chol_solve(fac_.data(), p_, b, x);
    return 0;
  }
  fac_.assign(A, A + pp);
  if (lu_inverse(fac_.data(), p_) != 0) {
    kind_ = 0;
    return 1;
  }
  kind_ = 2;  // fac_ holds inv(A): coefs = inv(A) * b as the reference does
  for (int64_t i = 0; i < p_; ++i) {
    double s = 0.0;
    for (int64_t k = 0; k < p_; ++k) s += fac_[i + k * p_] * b[k];
    x[i] = s;
  }
  return 0;
}

void Solver::inv_diag(double* d) const {
  if (kind_ == 1) {
    chol_inv_diag(fac_.data(), p_, d);
  } else if (kind_ == 2) {
    for (int64_t i = 0; i < p_; ++i) d[i] = fac_[i + i * p_];
  } else {
    for (int64_t i = 0; i < p_; ++i) d[i] = 0.0;
  }
}

void Solver::inverse(double* Ainv) const {
  if (kind_ == 1) {
    chol_inverse(fac_.data(), p_, Ainv);
  } else if (kind_ == 2) {
    std::memcpy(Ainv, fac_.data(), sizeof(double) * (size_t)(p_ * p_));
  }
}

}  // namespace sglm
