// Host build of the device Faddeeva/Voigt code, for CPU tests only (tests/test_faddeeva_host.py).
#include "../../prometheus_amd/csrc/faddeeva.h"
extern "C" {
void fad_re(long n, const double* x, const double* y, double* out) {
  for (long i = 0; i < n; ++i) out[i] = prom::faddeeva_re(x[i], y[i]);
}
void voigt(long n, const double* x, const double* s, const double* g, double* out) {
  for (long i = 0; i < n; ++i) out[i] = prom::voigt_profile(x[i], s[i], g[i]);
}
}
