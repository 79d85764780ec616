/* TEST INFRASTRUCTURE ONLY (the checker, never the product path): a C restatement of the molecular
 * line-of-sight optical depth, for full-size parity samples that the numpy oracle cannot finish in a test's
 * time (prom_oracle.molecular_sigma evaluates scipy's RegularGridInterpolator point by point: ~0.85 s per
 * wavelength on C5's 76,800 chords x 30 samples).
 *
 * Restates, for one molecular constituent:
 *   gasProperties.py:774-781  RegularGridInterpolator((P*10, T, 1/nu reversed), log10(xsec + offset),
 *                             bounds_error=False, fill_value=log10(offset)), method "linear"
 *   gasProperties.py:789-818  sigma = 10**rgi([clip(P, 1e-4), T, lambda]) - offset
 *   gasProperties.py:885-956  tau[c, w] += dx * sum_x chi * n[c, x] * sigma(P[c, x], T, shift[c] * wav[w])
 * with scipy 1.15's linear evaluation order (interpolate/_rgi.py _evaluate_linear: corners in
 * itertools.product order over (i, 1-y), (i+1, y) per dimension, weight = ((1*w_P)*w_T)*w_lam, value summed
 * from 0 in that order; find_indices: the interval i with grid[i] <= x < grid[i+1], clipped to [0, n-2];
 * out of bounds when x < grid[0] or x > grid[-1]).
 * Pinned against prom_oracle.molecular_sigma / optical_depth by tests/test_oracle_c.py.
 */
#include <math.h>
#include <stdint.h>

static int64_t interval(const double* g, int64_t n, double x) {
  /* largest i in [0, n-2] with g[i] <= x (x inside [g[0], g[n-1]]) */
  int64_t lo = 0, hi = n - 1;
  while (hi - lo > 1) {
    const int64_t m = (lo + hi) >> 1;
    if (g[m] <= x) lo = m; else hi = m;
  }
  return lo;
}

/* tau[c * nw + w] += dx * sum_x chi * n[c * nx + x] * sigma(P[c * nx + x], T, shift[c] * wav[w])
 * logsig: [np][nt][nl] = log10(xsec + offset) on the (P*10, T, lambda ascending) grid. */
void oracle_mol_tau(int64_t nc, int64_t nx, int64_t nw, const double* n, const double* P, const double* shift,
                    const double* wav, int64_t np_, const double* Pg, int64_t nt, const double* Tg, int64_t nl,
                    const double* lg, const double* logsig, double T, double offset, double chi, double dx,
                    double* tau) {
  const double fill = log10(offset);
  const int t_out = (T < Tg[0]) || (T > Tg[nt - 1]);
  const int64_t it = t_out ? 0 : interval(Tg, nt, T);
  const double yt = t_out ? 0.0 : (T - Tg[it]) / (Tg[it + 1] - Tg[it]);
  const double wt[2] = {1.0 - yt, yt};
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t c = 0; c < nc; ++c) {
    for (int64_t w = 0; w < nw; ++w) {
      const double lam = shift[c] * wav[w];
      const int l_out = (lam < lg[0]) || (lam > lg[nl - 1]);
      const int64_t il = l_out ? 0 : interval(lg, nl, lam);
      const double yl = l_out ? 0.0 : (lam - lg[il]) / (lg[il + 1] - lg[il]);
      const double wl[2] = {1.0 - yl, yl};
      double acc = 0.0;
      for (int64_t x = 0; x < nx; ++x) {
        double p = P[c * nx + x];
        if (p < 1e-4) p = 1e-4;
        double v;
        if (t_out || l_out || p < Pg[0] || p > Pg[np_ - 1]) {
          v = fill;
        } else {
          const int64_t ip = interval(Pg, np_, p);
          const double yp = (p - Pg[ip]) / (Pg[ip + 1] - Pg[ip]);
          const double wp[2] = {1.0 - yp, yp};
          v = 0.0;
          for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b)
              for (int d = 0; d < 2; ++d) {
                const double wgt = ((1.0 * wp[a]) * wt[b]) * wl[d];
                v = v + logsig[((ip + a) * nt + (it + b)) * nl + (il + d)] * wgt;
              }
        }
        acc += (chi * n[c * nx + x]) * (pow(10.0, v) - offset);
      }
      tau[c * nw + w] += acc * dx;
    }
  }
}
