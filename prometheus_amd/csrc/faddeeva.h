// Real part of the Faddeeva function w(z) = exp(-z^2) erfc(-iz), z = x + iy, y >= 0,
// and the Voigt profile built on it.
//
// Needed by the cross-section table kernel (AtmosphericConstituent.calculateVoigtProfile,
// reference gasProperties.py:672-692, which calls scipy.special.voigt_profile).  Only
// Re w is needed there.  Accuracy target: <= 1e-13 relative over the whole upper
// half plane that a line profile can produce (checked against mpmath in
// tests/test_faddeeva_host.py, and against scipy on the golden cross-section tables).
//
// Regions (x := |x| because Re w(-x+iy) = Re w(x+iy)):
//   A  x <  7, y <  YA    Taylor series in y about the real axis.  The real-axis
//                          derivatives come from exp(-x^2) (Hermite recurrence) and the
//                          Dawson function D and G = 1 - 2xD, both evaluated as
//                          exp(-x^2) times a positive power series (no cancellation).
//   B  x >= 7, y <  1     w = exp(-z^2) + (2i/sqrt(pi)) F(z), F the complex Dawson
//                          function from its asymptotic series; the error of Im F is
//                          proportional to y, like Re w itself.
//   C  |z| >= 7 otherwise  Laplace continued fraction.
//   D  remaining (|z| < 7, y >= YA): trapezoidal rule on the Voigt integral
//                          (y/pi) int exp(-t^2) / ((x-t)^2 + y^2) dt with a step that
//                          makes the pole term negligible.
#pragma once

#include <math.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define PROM_HD __host__ __device__ inline
#else
#define PROM_HD static inline
#endif

namespace prom {

constexpr double kSqrtPi = 1.7724538509055160273;
constexpr double kInvSqrtPi = 0.56418958354775628695;
constexpr double kTwoInvSqrtPi = 1.1283791670955125739;
constexpr double kPi = 3.14159265358979323846;
constexpr double kFaddeevaYA = 0.25;

// Dawson D(x) = exp(-x^2) S(x),  S = sum_n x^(2n+1) / (n! (2n+1))
// G(x) = 1 - 2x D(x) = exp(-x^2) (1 - T(x)),  T = sum_{n>=1} x^(2n) / (n! (2n-1))
PROM_HD void dawson_pair(double x, double e, double* D, double* G) {
  const double x2 = x * x;
  double p = 1.0;           // x^(2n) / n!
  double s = 1.0;           // sum p/(2n+1)
  double t = 0.0;           // sum_{n>=1} p/(2n-1)
  for (int n = 1; n < 400; ++n) {
    p *= x2 / n;
    const double ds = p / (2 * n + 1);
    s += ds;
    t += p / (2 * n - 1);
    if (n > x2 && ds < 1e-18 * s) break;
  }
  *D = e * (x * s);
  *G = e * (1.0 - t);
}

// Region A: Re w(x + iy), x < 7, small y.
PROM_HD double faddeeva_re_taylor(double x, double y) {
  const double e = exp(-x * x);
  double D, G;
  dawson_pair(x, e, &D, &G);
  // a_n: n-th derivative of exp(-x^2);  f_n: n-th derivative of D.
  double a_prev = e, a_cur = -2.0 * x * e;     // a_0, a_1
  double f_prev = D, f_cur = G;                // f_0, f_1
  double sum = e;                               // n = 0 term
  double yn = y;                                // y^n / n!
  double term = -kTwoInvSqrtPi * f_cur * yn;    // n = 1
  sum += term;
  int small = 0;
  for (int n = 1; n < 60; ++n) {
    // advance to derivative n+1
    const double a_next = -2.0 * x * a_cur - 2.0 * n * a_prev;
    const double f_next = -2.0 * x * f_cur - 2.0 * n * f_prev;
    a_prev = a_cur; a_cur = a_next;
    f_prev = f_cur; f_cur = f_next;
    const int m = n + 1;
    yn *= y / m;
    // Re[(a_m + i b_m) (iy)^m] / m!,  b_m = (2/sqrt(pi)) f_m
    switch (m & 3) {
      case 0: term = a_cur * yn; break;
      case 1: term = -kTwoInvSqrtPi * f_cur * yn; break;
      case 2: term = -a_cur * yn; break;
      default: term = kTwoInvSqrtPi * f_cur * yn; break;
    }
    sum += term;
    small = (fabs(term) < 1e-18 * fabs(sum)) ? small + 1 : 0;
    if (small >= 3) break;
  }
  return sum;
}

// Region B: x >= 7, y < 1.  Re w = Re exp(-z^2) - (2/sqrt(pi)) Im F(z),
// F(z) ~ sum_n c_n z^-(2n+1),  c_0 = 1/2, c_{n+1} = c_n (2n+1)/2.
PROM_HD double faddeeva_re_asym(double x, double y) {
  const double m2 = x * x + y * y;
  const double ur = x / m2, ui = -y / m2;              // 1/z
  const double vr = ur * ur - ui * ui, vi = 2.0 * ur * ui;  // 1/z^2
  double pr = ur, pi = ui;                             // z^-(2n+1)
  double c = 0.5;
  double sr = 0.0, si = 0.0;
  for (int n = 0; n < 200; ++n) {
    const double tr = c * pr, ti = c * pi;
    sr += tr;
    si += ti;
    if (fabs(tr) + fabs(ti) < 1e-18 * (fabs(sr) + fabs(si)) || (2.0 * n + 1.0) > 2.0 * m2) break;
    const double npr = pr * vr - pi * vi;
    const double npi = pr * vi + pi * vr;
    pr = npr; pi = npi;
    c *= (2.0 * n + 1.0) * 0.5;
  }
  const double ex = exp(y * y - x * x) * cos(2.0 * x * y);
  return ex - kTwoInvSqrtPi * si;
}

// Region C: Laplace continued fraction  w = (i/sqrt(pi)) / (z - (1/2)/(z - 1/(z - (3/2)/(z - ...))))
PROM_HD double faddeeva_re_cf(double x, double y) {
  const double az = sqrt(x * x + y * y);
  int nterm = (int)(12.0 + 260.0 / (az * az));
  if (nterm > 120) nterm = 120;
  double ur = x, ui = y;  // u = z
  for (int k = nterm; k >= 1; --k) {
    const double d = ur * ur + ui * ui;
    const double h = 0.5 * k / d;       // (k/2)/u = h * conj(u)
    ur = x - h * ur;
    ui = y + h * ui;
  }
  // w = i/(sqrt(pi) u) = i conj(u) / (sqrt(pi)|u|^2);  Re w = ui / (sqrt(pi)|u|^2)
  return kInvSqrtPi * ui / (ur * ur + ui * ui);
}

// Region D: trapezoidal rule on K(x,y) = (y/pi) int exp(-t^2)/((x-t)^2+y^2) dt.
PROM_HD double faddeeva_re_trapz(double x, double y) {
  double extra = y * y - x * x;
  if (extra < 0.0) extra = 0.0;
  double h = 2.0 * kPi * y / (40.0 + extra);
  if (h > 0.4) h = 0.4;
  const int nh = (int)(6.35 / h) + 1;
  const double y2 = y * y;
  double s = 0.0;
  for (int j = -nh; j <= nh; ++j) {
    const double t = j * h;
    const double d = x - t;
    s += exp(-t * t) / (d * d + y2);
  }
  return s * h * y / kPi;
}

PROM_HD double faddeeva_re(double x, double y) {
  x = fabs(x);
  if (x < 7.0) {
    if (y < kFaddeevaYA) return faddeeva_re_taylor(x, y);
    if (x * x + y * y >= 49.0) return faddeeva_re_cf(x, y);
    return faddeeva_re_trapz(x, y);
  }
  if (y < 1.0) return faddeeva_re_asym(x, y);
  return faddeeva_re_cf(x, y);
}

// scipy.special.voigt_profile(x, sigma, gamma) semantics (Faddeeva-based).
PROM_HD double voigt_profile(double x, double sigma, double gamma) {
  const double kInvSqrt2 = 0.707106781186547524401;
  const double kSqrt2Pi = 2.5066282746310002416123552393401042;
  if (sigma == 0.0) {
    if (gamma == 0.0) {
      if (x != x) return x;
      return x == 0.0 ? INFINITY : 0.0;
    }
    return gamma / kPi / (x * x + gamma * gamma);
  }
  if (gamma == 0.0) return 1.0 / kSqrt2Pi / sigma * exp(-(x / sigma) * (x / sigma) / 2.0);
  const double zr = x / sigma * kInvSqrt2;
  const double zi = gamma / sigma * kInvSqrt2;
  return faddeeva_re(zr, zi) / sigma / kSqrt2Pi;
}

}  // namespace prom
