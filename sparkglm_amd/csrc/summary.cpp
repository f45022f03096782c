// summary.cpp -- model-object arithmetic and printed summaries (host side).
//
// GLM.createObj (GLM.scala:59-88), GLM.summary (GLM.scala:998-1025), SummaryLM
// (LM.scala:66-137) and the print helpers sigDigits / roundDigits (utils.scala:146-169)
// are reproduced here so that every number a user of the reference reads comes out of
// the same C ABI, with Scala's Double.toString rendering.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "../../include/sglm.h"

namespace {

// java.lang.Math.round(double) -> long (floor(x + 0.5) with saturation; NaN -> 0)
long long java_round(double x) {
  if (std::isnan(x)) return 0;
  double f = std::floor(x + 0.5);
  if (f >= 9.2233720368547758e18) return std::numeric_limits<long long>::max();
  if (f <= -9.2233720368547758e18) return std::numeric_limits<long long>::min();
  return (long long)f;
}

// Double.toInt (Scala): truncation with saturation, NaN -> 0
int java_to_int(double x) {
  if (std::isnan(x)) return 0;
  if (x >= 2147483647.0) return 2147483647;
  if (x <= -2147483648.0) return -2147483647 - 1;
  return (int)x;
}

// java.lang.Double.toString: shortest round-trip digits; plain notation for
// 1e-3 <= |x| < 1e7, computerized scientific notation ("1.0E-4") otherwise.
std::string java_double(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
  if (x == 0.0) return std::signbit(x) ? "-0.0" : "0.0";
  char buf[64];
  int prec = 0;
  for (prec = 0; prec < 17; ++prec) {
    std::snprintf(buf, sizeof buf, "%.*e", prec, x);
    if (std::strtod(buf, nullptr) == x) break;
  }
  // buf = [-]d.ddddde[+-]XX
  std::string s(buf);
  bool neg = s[0] == '-';
  if (neg) s = s.substr(1);
  size_t epos = s.find('e');
  int exp10 = std::atoi(s.c_str() + epos + 1);
  std::string digits;
  for (size_t i = 0; i < epos; ++i)
    if (s[i] != '.') digits.push_back(s[i]);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  std::string out = neg ? "-" : "";
  const double ax = std::fabs(x);
  if (ax >= 1e-3 && ax < 1e7) {
    const int ip = exp10 + 1;  // digits before the point
    if (ip <= 0) {
      out += "0.";
      out += std::string((size_t)(-ip), '0');
      out += digits;
    } else if ((size_t)ip >= digits.size()) {
      out += digits + std::string((size_t)ip - digits.size(), '0') + ".0";
    } else {
      out += digits.substr(0, (size_t)ip) + "." + digits.substr((size_t)ip);
    }
  } else {
    out += digits.substr(0, 1) + ".";
    out += digits.size() > 1 ? digits.substr(1) : std::string("0");
    out += "E" + std::to_string(exp10);
  }
  return out;
}

double sig_digits(double num, int digits) {  // utils.scala:154-169
  if (num == 0) return 0.0;
  const double absNum = std::fabs(num);
  const double d = std::ceil(std::log10(absNum));
  const int power = java_to_int((double)digits - d);
  const double magnitude = std::pow(10.0, power);
  const long long shifted = java_round(absNum * magnitude);
  if (num > 0) return (double)shifted / magnitude;
  return -1.0 * (double)shifted / magnitude;
}

double round_digits(double num, int digits) {  // utils.scala:146-149
  const long long top = java_round(num * std::pow(10.0, digits));
  return (double)top / std::pow(10.0, digits);
}

double norm_cdf(double x) { return 0.5 * (1.0 + std::erf(x / std::sqrt(2.0))); }

// Regularized incomplete beta I_x(a,b) by Lentz's continued fraction.
double betacf(double a, double b, double x) {
  const double tiny = 1e-300, eps = 1e-16;
  double qab = a + b, qap = a + 1.0, qam = a - 1.0, c = 1.0, d = 1.0 - qab * x / qap;
  if (std::fabs(d) < tiny) d = tiny;
  d = 1.0 / d;
  double h = d;
  for (int m = 1; m <= 10000; ++m) {
    const int m2 = 2 * m;
    double aa = m * (b - m) * x / ((qam + m2) * (a + m2));
    d = 1.0 + aa * d;
    if (std::fabs(d) < tiny) d = tiny;
    c = 1.0 + aa / c;
    if (std::fabs(c) < tiny) c = tiny;
    d = 1.0 / d;
    h *= d * c;
    aa = -(a + m) * (qab + m) * x / ((a + m2) * (qap + m2));
    d = 1.0 + aa * d;
    if (std::fabs(d) < tiny) d = tiny;
    c = 1.0 + aa / c;
    if (std::fabs(c) < tiny) c = tiny;
    d = 1.0 / d;
    const double del = d * c;
    h *= del;
    if (std::fabs(del - 1.0) < eps) break;
  }
  return h;
}

double ibeta(double a, double b, double x) {
  if (x <= 0.0) return 0.0;
  if (x >= 1.0) return 1.0;
  const double lbt = std::lgamma(a + b) - std::lgamma(a) - std::lgamma(b) + a * std::log(x) + b * std::log1p(-x);
  const double bt = std::exp(lbt);
  if (x < (a + 1.0) / (a + b + 2.0)) return bt * betacf(a, b, x) / a;
  return 1.0 - bt * betacf(b, a, 1.0 - x) / b;
}

// StudentsT(df).cdf(t)
double t_cdf(double t, double df) {
  const double x = df / (df + t * t);
  const double tail = 0.5 * ibeta(df / 2.0, 0.5, x);
  return t >= 0 ? 1.0 - tail : tail;
}

std::string fmt5(const char* a, const std::string& b, const std::string& c, const std::string& d, const std::string& e) {
  char buf[512];
  std::snprintf(buf, sizeof buf, "%-12s %12s %12s %12s %12s", a, b.c_str(), c.c_str(), d.c_str(), e.c_str());
  return buf;
}

int64_t emit(const std::string& s, char* buf, int64_t buflen) {
  const int64_t need = (int64_t)s.size() + 1;
  if (buf && buflen > 0) {
    const int64_t k = need <= buflen ? need - 1 : buflen - 1;
    std::memcpy(buf, s.data(), (size_t)k);
    buf[k] = '\0';
  }
  return need;
}

}  // namespace

extern "C" {

double sglm_sig_digits(double num, int digits) { return sig_digits(num, digits); }
double sglm_round_digits(double num, int digits) { return round_digits(num, digits); }
int64_t sglm_java_double_string(double x, char* buf, int64_t buflen) { return emit(java_double(x), buf, buflen); }
double sglm_pval_normal(double z) { return 2.0 * (1.0 - norm_cdf(std::fabs(z))); }
double sglm_pval_t(double t, double df) { return 2.0 * (1.0 - t_cdf(std::fabs(t), df)); }

int sglm_glm_create_obj(const sglm_preglm* pre, int64_t p, sglm_glm_derived* out) {
  if (!pre || !out) return SGLM_EINVAL;
  const double nrow = pre->nrow;  // y.count (GLM.scala:65)
  out->df_residual = nrow - (double)p;
  out->df_null = nrow - 1.0;
  out->p_dispersion = pre->pearson / out->df_residual;
  out->aic = -2.0 * pre->loglik + 2.0 * (double)p;
  return SGLM_OK;
}

int64_t sglm_glm_summary(const sglm_preglm* pre, int64_t p, const char* const* xnames, const char* yname,
                         const char* family, const char* link, char* buf, int64_t buflen) {
  if (!pre || !xnames || p <= 0) return -1;
  sglm_glm_derived dd;
  sglm_glm_create_obj(pre, p, &dd);
  const int dfNDev = java_to_int(pre->nrow) - 1;
  const int dfDev = java_to_int(pre->nrow) - (int)p;
  std::string f = xnames[0];
  for (int64_t i = 1; i < p; ++i) f += std::string(" + ") + xnames[i];
  std::string s;
  s += "Model:\n";
  s += std::string(yname ? yname : "y") + " ~ " + f + "\n";
  s += std::string("Family: ") + (family ? family : "") + "\n";
  s += std::string("Link: ") + (link ? link : "") + "\n";
  s += "\n\n";
  s += "Coefficients:\n";
  s += fmt5("", "Estimate", "Std. Error", "z value", "Pr(>|z|)") + "\n";
  for (int64_t i = 0; i < p; ++i) {
    const double c = pre->coefs[i], se = pre->std_err[i], z = c / se;
    const double pv = 2.0 * (1.0 - norm_cdf(std::fabs(z)));
    s += fmt5(xnames[i], java_double(sig_digits(c, 6)), java_double(sig_digits(se, 6)),
              java_double(sig_digits(z, 6)), java_double(sig_digits(pv, 6))) +
         "\n";
  }
  s += "\n\n";
  s += "Null deviance: " + java_double(sig_digits(pre->null_deviance, 6)) + " on " + std::to_string(dfNDev) +
       " degress of freedom\n";
  s += "Residual deviance: " + java_double(sig_digits(pre->deviance, 6)) + " on " + std::to_string(dfDev) +
       " degress of freedom\n";
  s += "AIC: " + java_double(sig_digits(dd.aic, 5)) + "\n";
  s += "\n\n";
  s += "Number of Fisher Scoring iterations: " + std::to_string(pre->iter) + "\n";
  return emit(s, buf, buflen);
}

int64_t sglm_lm_summary(const sglm_prelm* pre, int64_t p, const char* const* xnames, const char* yname, char* buf,
                        int64_t buflen) {
  if (!pre || !xnames || p <= 0) return -1;
  const double nrow = pre->nrow;
  const double adjR2 = 1.0 - (((1.0 - pre->r2) * (nrow - 1.0)) / (nrow - (double)p - 1.0));  // LM.scala:68-70
  const double dfm = (double)(p - 1);                                                        // LM.scala:72-74
  const double dfe = (double)(java_to_int(nrow) - (int)p);                                   // LM.scala:76-78
  std::string f = xnames[0];
  for (int64_t i = 1; i < p; ++i) f += std::string(" + ") + xnames[i];
  std::string s;
  s += "Model:\n";
  s += std::string(yname ? yname : "y") + " ~ " + f + "\n\n";
  s += "Coefficients:\n";
  s += fmt5("", "Estimate", "Std. Error", "t value", "Pr(>|t|)");
  for (int64_t i = 0; i < p; ++i) {
    const double c = pre->coefs[i], se = pre->std_err[i], t = c / se;
    const double pv = 2.0 * (1.0 - t_cdf(std::fabs(t), dfe));
    s += "\n" + fmt5(xnames[i], java_double(sig_digits(c, 6)), java_double(sig_digits(se, 6)),
                     java_double(sig_digits(t, 6)), java_double(sig_digits(pv, 6)));
  }
  s += "\n\n";
  s += "Residual standard error: " + java_double(sig_digits(pre->sigma, 6)) + " on " + java_double(dfe) +
       " degrees of freedom\n\n";
  s += "Multiple R-Squared: " + java_double(round_digits(pre->r2, 4)) + ", Adusted R-Squared: " +
       java_double(round_digits(adjR2, 4)) + "\n\n";
  s += "F-statistic: " + java_double(sig_digits(pre->fstat, 5)) + " on " + java_double(dfm) + " and " +
       java_double(dfe) + " DF\n\n";
  return emit(s, buf, buflen);
}

}  // extern "C"
