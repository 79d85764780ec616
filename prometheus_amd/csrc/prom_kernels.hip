// HIP kernels for gfx950 (MI355X).  Compiled with -ffp-contract=off: every product and sum below
// is rounded exactly where the numpy reference rounds it (no silent FMA contraction); FMAs appear
// only inside the ocml transcendentals, as in any libm.
//
// Kernels (reference functions they restate):
//   k_table_lookup   n_interp_log / getSigmaAbs              gasProperties.py:34-51, :727-735
//   k_voigt          calculateVoigtProfile (+ log10 table)   gasProperties.py:672-715
//   k_density        calculateNumberDensity (all scenarios)  gasProperties.py:143-516
//   k_mol_sigma      MolecularConstituent.getSigmaAbs        gasProperties.py:789-818
//   transit pipeline Transit.sumOverChords + getLOSopticalDepth_Batch (gasProperties.py:885-956,
//                    :1160-1258):
//     k_ntot      n(c, x) for every scenario, chord and line-of-sight sample
//     k_columns   blocking masks, column densities N = sum_x(n chi) dx (numpy pairwise order),
//                 tau upper bound per chord -> active / transparent / blocked
//     k_compact   per phase, in chord order: packed records of the active chords, transparent
//                 and total F_out sums
//     k_sigma     sigma[s][o][w] = 10^interp(shift_o * lambda_w) - offset  (HBM-streaming)
//     k_tau<NS>   per (phase, wavelength): tau over active chords, exp(-tau), disk sum, ratio
#include "faddeeva.h"
#include "prom_internal.h"

namespace prom {

constexpr int kBlock = 256;

static inline unsigned grid_for(int64_t n, int block = kBlock, int64_t cap = 1 << 20) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// numpy.interp (numpy/_core/src/multiarray/compiled_base.c arr_interp) for one target.
__device__ __forceinline__ double np_interp(double t, const double* __restrict__ xp,
                                            const double* __restrict__ fp, int64_t n) {
  if (t != t) return t;
  if (n == 1) return (t < xp[0]) ? fp[0] : fp[0];
  if (t < xp[0]) return fp[0];
  if (t > xp[n - 1]) return fp[n - 1];
  if (t == xp[n - 1]) return fp[n - 1];
  int64_t lo = 0, hi = n - 1;  // xp[lo] <= t < xp[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (xp[mid] <= t) lo = mid; else hi = mid;
  }
  if (xp[lo] == t) return fp[lo];
  const double slope = (fp[lo + 1] - fp[lo]) / (xp[lo + 1] - xp[lo]);
  double r = slope * (t - xp[lo]) + fp[lo];
  if (r != r) {
    r = slope * (t - xp[lo + 1]) + fp[lo + 1];
    if (r != r && fp[lo] == fp[lo + 1]) r = fp[lo];
  }
  return r;
}

// numpy.heaviside(d, 1.0)
__device__ __forceinline__ double heaviside1(double d) { return d < 0.0 ? 0.0 : (d >= 0.0 ? 1.0 : d); }

// One density sample, in the reference's evaluation order (see prom_density_kind in prom_hip.h).
__device__ __forceinline__ double density_at(const DensityDev& m, double xv, double y, double z,
                                             double bx, double by) {
  const double dx = xv - bx, dy = y - by;
  switch (m.kind) {
    case PROM_DENSITY_BAROMETRIC: {
      const double r = sqrt((dx * dx + dy * dy) + z * z);
      return (m.p[0] * exp((m.p[1] - r) / m.p[2])) * heaviside1(r - m.p[1]);
    }
    case PROM_DENSITY_HYDROSTATIC: {
      const double r = sqrt((dx * dx + dy * dy) + z * z);
      const double jeans = m.p[2] / (m.p[3] * r) * heaviside1(r - m.p[1]);
      return m.p[0] * exp(jeans - m.p[4]);
    }
    case PROM_DENSITY_POWERLAW: {
      const double r = sqrt((dx * dx + dy * dy) + z * z);
      return (m.p[0] * pow(m.p[1] / r, m.p[2])) * heaviside1(r - m.p[1]);
    }
    case PROM_DENSITY_TORUS: {
      const double a = sqrt(dx * dx + dy * dy);
      const double ta = (a - m.p[1]) / m.p[2];
      const double tz = z / m.p[3];
      return m.p[0] * (exp(-(ta * ta)) * exp(-(tz * tz)));
    }
    default:
      return __builtin_nan("");
  }
}

// numpy pairwise_sum of (a[i] * chi) for i < n (numpy/_core/src/umath/loops_utils.h.src),
// then the reduction identity: 0.0 + result.
__device__ __forceinline__ double pw_leaf(const double* __restrict__ a, int64_t n, double chi) {
  if (n < 8) {
    double r = 0.0;
    for (int64_t i = 0; i < n; ++i) r += a[i] * chi;
    return r;
  }
  double r0 = a[0] * chi, r1 = a[1] * chi, r2 = a[2] * chi, r3 = a[3] * chi;
  double r4 = a[4] * chi, r5 = a[5] * chi, r6 = a[6] * chi, r7 = a[7] * chi;
  int64_t i = 8;
  const int64_t lim = n - (n % 8);
  for (; i < lim; i += 8) {
    r0 += a[i + 0] * chi; r1 += a[i + 1] * chi; r2 += a[i + 2] * chi; r3 += a[i + 3] * chi;
    r4 += a[i + 4] * chi; r5 += a[i + 5] * chi; r6 += a[i + 6] * chi; r7 += a[i + 7] * chi;
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += a[i] * chi;
  return res;
}

__device__ double pairwise_sum_chi(const double* __restrict__ a, int64_t n, double chi) {
  if (n <= 128) return 0.0 + pw_leaf(a, n, chi);
  struct Frame { int64_t off, n; int stage; double left; };
  Frame st[48];
  int sp = 0;
  st[0] = {0, n, 0, 0.0};
  double ret = 0.0;
  while (sp >= 0) {
    Frame& f = st[sp];
    if (f.n <= 128) { ret = pw_leaf(a + f.off, f.n, chi); --sp; continue; }
    int64_t n2 = f.n / 2;
    n2 -= n2 % 8;
    if (f.stage == 0) { f.stage = 1; st[++sp] = {f.off, n2, 0, 0.0}; }
    else if (f.stage == 1) { f.left = ret; f.stage = 2; st[++sp] = {f.off + n2, f.n - n2, 0, 0.0}; }
    else { ret = f.left + ret; --sp; }
  }
  return 0.0 + ret;
}

// ------------------------------------------------------------------ function-level kernels
__global__ void k_table_lookup(const double* __restrict__ xp, const double* __restrict__ fp, int64_t n,
                               double offset, const double* __restrict__ t, int64_t nt,
                               double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nt;
       i += (int64_t)gridDim.x * blockDim.x) {
    out[i] = pow(10.0, np_interp(t[i], xp, fp, n)) - offset;
  }
}

void launch_table_lookup(hipStream_t s, const double* x, const double* y, int64_t n, double offset,
                         const double* targets, int64_t nt, double* out) {
  if (nt == 0) return;
  hipLaunchKernelGGL(k_table_lookup, dim3(grid_for(nt)), dim3(kBlock), 0, s, x, y, n, offset, targets,
                     nt, out);
  PROM_HIP(hipGetLastError());
}

__global__ void k_voigt(const double* __restrict__ x, int64_t n, const double* __restrict__ lw,
                        const double* __restrict__ lg, const double* __restrict__ lc, int32_t nl,
                        double sigma_v, double c_light, double offset, int log_table,
                        double* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double cx = c_light / x[i];
    double s = 0.0;
    for (int32_t l = 0; l < nl; ++l) {
      const double lam0 = lw[l];
      const double prof = voigt_profile(cx - c_light / lam0, sigma_v / lam0, lg[l]);
      s += lc[l] * prof;
    }
    out[i] = log_table ? log10(s + offset) : s;
  }
}

void launch_voigt(hipStream_t s, const double* x, int64_t n, const double* lw, const double* lg,
                  const double* lc, int32_t nl, double sigma_v, double c_light, double offset,
                  int log_table, double* out) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_voigt, dim3(grid_for(n, 128)), dim3(128), 0, s, x, n, lw, lg, lc, nl, sigma_v,
                     c_light, offset, log_table, out);
  PROM_HIP(hipGetLastError());
}

__global__ void k_density(DensityDev m, const double* __restrict__ x, int32_t n_x,
                          const double* __restrict__ y, const double* __restrict__ z,
                          const double* __restrict__ bx, const double* __restrict__ by, int64_t n_chords,
                          double* __restrict__ out) {
  const int64_t tot = n_chords * n_x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = i / n_x;
    const int32_t ix = (int32_t)(i - c * n_x);
    out[i] = density_at(m, x[ix], y[c], z[c], bx[c], by[c]);
  }
}

void launch_density(hipStream_t s, const DensityDev& m, const double* x, int32_t n_x, const double* y,
                    const double* z, const double* bx, const double* by, int64_t n_chords,
                    double* out) {
  if (n_chords * n_x == 0) return;
  hipLaunchKernelGGL(k_density, dim3(grid_for(n_chords * n_x)), dim3(kBlock), 0, s, m, x, n_x, y, z, bx,
                     by, n_chords, out);
  PROM_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ molecular lookup
// Bracketing index of a sorted axis for RegularGridInterpolator (scipy _find_indices):
// i = searchsorted(g, v) - 1 clipped to [0, n-2]; t = (v - g[i]) / (g[i+1] - g[i]).
// Returns false when v is outside [g[0], g[n-1]] (fill value).
__device__ __forceinline__ bool rgi_bracket(const double* __restrict__ g, int64_t n, double v, int64_t* i,
                                            double* t) {
  if (!(v >= g[0] && v <= g[n - 1])) return false;
  int64_t lo = 0, hi = n;  // first index with g[idx] >= v  (searchsorted left)
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (g[mid] < v) lo = mid + 1; else hi = mid;
  }
  int64_t k = lo - 1;
  if (k < 0) k = 0;
  if (k > n - 2) k = n - 2;
  *i = k;
  *t = (v - g[k]) / (g[k + 1] - g[k]);
  return true;
}

// Trilinear value at (P, T, w), scipy's hypercube order: corners (dP, dT, dw) lexicographic,
// weight = ((1 * wP) * wT) * ww, value = ((0 + v000 w) + v001 w) + ...
__device__ __forceinline__ double mol_value(const double* __restrict__ V, int32_t n_t, int64_t n_w,
                                            int64_t ip, double tp, int64_t it, double tt, int64_t iw,
                                            double tw) {
  double value = 0.0;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int dp = (c >> 2) & 1, dt = (c >> 1) & 1, dw = c & 1;
    const double wp = dp ? tp : 1.0 - tp;
    const double wt = dt ? tt : 1.0 - tt;
    const double ww = dw ? tw : 1.0 - tw;
    const double weight = ((1.0 * wp) * wt) * ww;
    value = value + V[((ip + dp) * n_t + (it + dt)) * n_w + (iw + dw)] * weight;
  }
  return value;
}

__global__ void k_mol_sigma(const double* __restrict__ Pg, int32_t n_p, const double* __restrict__ Tg,
                            int32_t n_t, const double* __restrict__ Wg, int64_t n_w,
                            const double* __restrict__ V, double offset, int64_t n_chords, int32_t n_x,
                            const double* __restrict__ P, double T, int64_t n_wav,
                            const double* __restrict__ wav, double* __restrict__ out) {
  const int64_t tot = n_chords * n_x * n_wav;
  const double fill = log10(offset);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < tot;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t w = i % n_wav;
    const int64_t cx = i / n_wav;
    const int64_t c = cx / n_x;
    double p = P[cx];
    p = p < 1e-4 ? 1e-4 : p;
    int64_t ip, it, iw;
    double tp, tt, tw;
    double v = fill;
    if (rgi_bracket(Pg, n_p, p, &ip, &tp) && rgi_bracket(Tg, n_t, T, &it, &tt) &&
        rgi_bracket(Wg, n_w, wav[c * n_wav + w], &iw, &tw))
      v = mol_value(V, n_t, n_w, ip, tp, it, tt, iw, tw);
    out[i] = pow(10.0, v) - offset;
  }
}

void launch_molecular_sigma(hipStream_t s, const MolTable& t, int64_t n_chords, int32_t n_x,
                            const double* P, double T, int64_t n_wav, const double* wav, double* out) {
  const int64_t tot = n_chords * n_x * n_wav;
  if (tot == 0) return;
  hipLaunchKernelGGL(k_mol_sigma, dim3(grid_for(tot)), dim3(kBlock), 0, s, t.P.as<double>(), t.n_p,
                     t.T.as<double>(), t.n_t, t.W.as<double>(), t.n_w, t.V.as<double>(), t.offset,
                     n_chords, n_x, P, T, n_wav, wav, out);
  PROM_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ reductions
__global__ void k_max(const double* __restrict__ v, int64_t n, double* __restrict__ out) {
  __shared__ double sm[kBlock];
  double m = -INFINITY;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const double a = v[i];
    m = (a > m || a != a) ? a : m;
  }
  sm[threadIdx.x] = m;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      const double a = sm[threadIdx.x + s];
      if (a > sm[threadIdx.x] || a != a) sm[threadIdx.x] = a;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sm[0];
}

double reduce_max(hipStream_t s, const double* v, int64_t n, double* scratch_dev) {
  hipLaunchKernelGGL(k_max, dim3(1), dim3(kBlock), 0, s, v, n, scratch_dev);
  PROM_HIP(hipGetLastError());
  double h = 0.0;
  PROM_HIP(hipMemcpyAsync(&h, scratch_dev, sizeof(double), hipMemcpyDeviceToHost, s));
  PROM_HIP(hipStreamSynchronize(s));
  return h;
}

// ------------------------------------------------------------------ transit pipeline
__global__ void k_ntot(DensityDev m, int32_t sc, const double* __restrict__ x, int32_t n_x,
                       const double* __restrict__ cy, const double* __restrict__ cz, int32_t n_pr,
                       int32_t n_orb, const double* __restrict__ bx, const double* __restrict__ by,
                       const double* __restrict__ tab, double* __restrict__ ntot) {
  const int64_t per = (int64_t)n_orb * n_pr * n_x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < per;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t ix = (int32_t)(i % n_x);
    const int64_t c = i / n_x;
    const int32_t ip = (int32_t)(c % n_pr);
    const int32_t o = (int32_t)(c / n_pr);
    double v;
    if (m.kind == PROM_DENSITY_TABULATED)
      v = tab[((int64_t)ip * n_orb + o) * n_x + ix];
    else
      v = density_at(m, x[ix], cy[ip], cz[ip], bx[sc * n_orb + o], by[sc * n_orb + o]);
    ntot[(int64_t)sc * per + i] = v;
  }
}

__global__ void k_columns(const TermDev* __restrict__ terms, int32_t n_terms,
                          const double* __restrict__ ntot, int32_t n_x, int32_t n_pr, int32_t n_orb,
                          double delta_x, const double* __restrict__ cy, const double* __restrict__ cz,
                          const double* __restrict__ planet_y, double planet_R, int32_t n_moons,
                          const double* __restrict__ moon_y, const double* __restrict__ moon_R,
                          const double* __restrict__ sig_max, double mol_max_any, double cull,
                          double* __restrict__ ncol, double* __restrict__ molcol,
                          int32_t* __restrict__ flags) {
  const int64_t nc = (int64_t)n_orb * n_pr;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < nc;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int32_t ip = (int32_t)(c % n_pr);
    const int32_t o = (int32_t)(c / n_pr);
    const double y = cy[ip], z = cz[ip];
    // gasProperties.py:1224-1230
    const double dyp = y - planet_y[o];
    bool blocked = sqrt(dyp * dyp + z * z) < planet_R;
    for (int32_t m = 0; m < n_moons; ++m) {
      const double dym = y - moon_y[m * n_orb + o];
      blocked = blocked || ((dym * dym + z * z) < moon_R[m] * moon_R[m]);
    }
    if (blocked) {
      for (int32_t t = 0; t < n_terms; ++t)
        if (!terms[t].is_molecule) ncol[((int64_t)terms[t].slot * n_orb + o) * n_pr + ip] = 0.0;
      flags[c] = 2;
      continue;
    }
    double bound = 0.0;
    for (int32_t t = 0; t < n_terms; ++t) {
      const TermDev td = terms[t];
      const double* row = ntot + (((int64_t)td.scenario * n_orb + o) * n_pr + ip) * n_x;
      if (!td.is_molecule) {
        // gasProperties.py:940  np.sum(n_tot * chi, axis=1) * delta_x
        const double N = pairwise_sum_chi(row, n_x, td.chi) * delta_x;
        ncol[((int64_t)td.slot * n_orb + o) * n_pr + ip] = N;
        bound += N * sig_max[td.slot];
      } else {
        double s = 0.0;
        for (int32_t ix = 0; ix < n_x; ++ix) s += row[ix] * td.chi;
        s *= delta_x;
        molcol[((int64_t)td.slot * n_orb + o) * n_pr + ip] = s;
        bound += s * mol_max_any;
      }
    }
    flags[c] = (bound <= cull) ? 1 : 0;  // NaN bound stays active, like the reference
  }
}

// One workgroup per phase: stream compaction of the active chords in chord order.
__global__ void __launch_bounds__(kBlock) k_compact(const int32_t* __restrict__ flags,
                                                    const double* __restrict__ fout,
                                                    const double* __restrict__ ncol, int32_t n_atoms,
                                                    int32_t n_pr, int32_t n_orb,
                                                    double* __restrict__ recs,
                                                    int32_t* __restrict__ act_ip,
                                                    int32_t* __restrict__ counts,
                                                    double* __restrict__ tsum,
                                                    double* __restrict__ fsum) {
  const int32_t o = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __shared__ int32_t wcount[kBlock / 64];
  __shared__ double red[2][kBlock];
  int32_t base = 0, ntr = 0, nbl = 0;
  double tpart = 0.0, fpart = 0.0;
  const int32_t stride = 1 + n_atoms;
  for (int32_t chunk = 0; chunk < n_pr; chunk += kBlock) {
    const int32_t ip = chunk + threadIdx.x;
    const int32_t f = ip < n_pr ? flags[(int64_t)o * n_pr + ip] : 3;
    if (ip < n_pr) {
      const double fo = fout[ip];
      fpart += fo;
      if (f == 1) { tpart += fo; ++ntr; }
      if (f == 2) ++nbl;
    }
    const bool act = (f == 0);
    const unsigned long long mask = __ballot(act);
    const int32_t before = __popcll(mask & ((1ull << lane) - 1ull));
    if (lane == 0) wcount[wid] = __popcll(mask);
    __syncthreads();
    int32_t wbase = 0, tot = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
      if (w < wid) wbase += wcount[w];
      tot += wcount[w];
    }
    if (act) {
      const int32_t pos = base + wbase + before;
      act_ip[(int64_t)o * n_pr + pos] = ip;
      double* r = recs + ((int64_t)o * n_pr + pos) * stride;
      r[0] = fout[ip];
      for (int32_t s = 0; s < n_atoms; ++s) r[1 + s] = ncol[((int64_t)s * n_orb + o) * n_pr + ip];
    }
    base += tot;
    __syncthreads();
  }
  red[0][threadIdx.x] = tpart;
  red[1][threadIdx.x] = fpart;
  __shared__ int32_t cnt[2][kBlock];
  cnt[0][threadIdx.x] = ntr;
  cnt[1][threadIdx.x] = nbl;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
      cnt[0][threadIdx.x] += cnt[0][threadIdx.x + s];
      cnt[1][threadIdx.x] += cnt[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    tsum[o] = red[0][0];
    fsum[o] = red[1][0];
    counts[o * 3 + 0] = base;
    counts[o * 3 + 1] = cnt[0][0];
    counts[o * 3 + 2] = cnt[1][0];
  }
}

// sigma[slot][o][w] = 10^interp(shift[o] * lambda[w]) - offset     (gasProperties.py:916-917, :941-953)
__global__ void k_sigma(const double* __restrict__ xp, const double* __restrict__ fp, int64_t n,
                        double offset, const double* __restrict__ shift, const double* __restrict__ wav,
                        int64_t n_wav, double* __restrict__ sig) {
  const int32_t o = blockIdx.y;
  const double s = shift[o];
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < n_wav;
       w += (int64_t)gridDim.x * blockDim.x) {
    sig[(int64_t)o * n_wav + w] = pow(10.0, np_interp(s * wav[w], xp, fp, n)) - offset;
  }
}

// Fused tau -> exp(-tau) -> disk sum -> ratio.  One thread per (phase o, wavelength w); the chord
// loop is uniform across the workgroup (all threads share the phase), so the packed chord records
// are read with scalar loads.  NS = number of atomic constituents (0 = runtime count via LDS).
template <int NS>
__global__ void __launch_bounds__(kBlock) k_tau(const double* __restrict__ sig,
                                                const double* __restrict__ recs,
                                                const int32_t* __restrict__ counts,
                                                const double* __restrict__ tsum,
                                                const double* __restrict__ fsum, int32_t n_atoms_rt,
                                                int32_t n_pr, int32_t n_orb, int64_t n_wav,
                                                double* __restrict__ R) {
  const int32_t o = blockIdx.y;
  const int64_t w = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  const bool live = w < n_wav;
  const int64_t wc = live ? w : n_wav - 1;
  const int32_t n_act = counts[o * 3];
  double acc = 0.0;
  if constexpr (NS > 0) {
    constexpr int stride = 1 + NS;
    double sg[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) sg[s] = sig[((int64_t)s * n_orb + o) * n_wav + wc];
    const double* __restrict__ rec = recs + (int64_t)o * n_pr * stride;
    for (int32_t i = 0; i < n_act; ++i) {
      const double* r = rec + (int64_t)i * stride;
      double tau = r[1] * sg[0];
#pragma unroll
      for (int s = 1; s < NS; ++s) tau = tau + r[1 + s] * sg[s];
      acc = acc + r[0] * exp(-tau);
    }
  } else {
    extern __shared__ double sgl[];  // [n_atoms][kBlock]
    const int32_t ns = n_atoms_rt;
    const int32_t stride = 1 + ns;
    for (int32_t s = 0; s < ns; ++s) sgl[s * kBlock + threadIdx.x] = sig[((int64_t)s * n_orb + o) * n_wav + wc];
    const double* __restrict__ rec = recs + (int64_t)o * n_pr * stride;
    for (int32_t i = 0; i < n_act; ++i) {
      const double* r = rec + (int64_t)i * stride;
      double tau = r[1] * sgl[threadIdx.x];
      for (int32_t s = 1; s < ns; ++s) tau = tau + r[1 + s] * sgl[s * kBlock + threadIdx.x];
      acc = acc + r[0] * exp(-tau);
    }
  }
  if (live) R[(int64_t)o * n_wav + w] = (acc + tsum[o]) / fsum[o];
}

void launch_transit(hipStream_t s, TransitDev& tr, const std::vector<AtomTable>& tables,
                    const std::vector<MolTable>& mtables, hipEvent_t* ev, int* variant) {
  const int64_t per = (int64_t)tr.n_orb * tr.n_pr * tr.n_x;
  PROM_HIP(hipEventRecord(ev[0], s));
  // 1. densities
  for (int32_t sc = 0; sc < tr.n_sc; ++sc) {
    const DensityDev& m = tr.dens[sc];
    const double* tab = nullptr;
    if (m.kind == PROM_DENSITY_TABULATED) tab = tr.tab.as<double>() + tr.tab_off[sc];
    hipLaunchKernelGGL(k_ntot, dim3(grid_for(per)), dim3(kBlock), 0, s, m, sc, tr.x.as<double>(), tr.n_x,
                       tr.cy.as<double>(), tr.cz.as<double>(), tr.n_pr, tr.n_orb, tr.body_x.as<double>(),
                       tr.body_y.as<double>(), tab, tr.ntot.as<double>());
    PROM_HIP(hipGetLastError());
  }
  double mol_max = 0.0;
  for (const auto& t : tr.terms)
    if (t.is_molecule) mol_max = std::max(mol_max, std::pow(10.0, mtables[t.table].vmax));
  const int64_t nc = (int64_t)tr.n_orb * tr.n_pr;
  hipLaunchKernelGGL(k_columns, dim3(grid_for(nc, 64)), dim3(64), 0, s, tr.terms_dev.as<TermDev>(),
                     tr.n_terms, tr.ntot.as<double>(), tr.n_x, tr.n_pr, tr.n_orb, tr.delta_x,
                     tr.cy.as<double>(), tr.cz.as<double>(), tr.planet_y.as<double>(), tr.planet_R,
                     tr.n_moons, tr.moon_y.as<double>(), tr.moon_R.as<double>(),
                     tr.sigma_max_dev.as<double>(), mol_max, tr.cull_tau, tr.ncol.as<double>(),
                     tr.molcol.as<double>(), tr.flags.as<int32_t>());
  PROM_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_compact, dim3(tr.n_orb), dim3(kBlock), 0, s, tr.flags.as<int32_t>(),
                     tr.cfout.as<double>(), tr.ncol.as<double>(), tr.n_atoms, tr.n_pr, tr.n_orb,
                     tr.recs.as<double>(), tr.act_ip.as<int32_t>(), tr.counts.as<int32_t>(),
                     tr.tsum.as<double>(), tr.fsum.as<double>());
  PROM_HIP(hipGetLastError());
  PROM_HIP(hipEventRecord(ev[1], s));
  // 2. sigma resample
  for (const auto& t : tr.terms) {
    if (t.is_molecule) continue;
    const AtomTable& tb = tables[t.table];
    dim3 g(grid_for(tr.n_wav, kBlock, 65535), tr.n_orb);
    hipLaunchKernelGGL(k_sigma, g, dim3(kBlock), 0, s, tb.x.as<double>(), tb.y.as<double>(), tb.n, tb.offset,
                       tr.shift.as<double>() + (int64_t)t.scenario * tr.n_orb, tr.wav.as<double>(), tr.n_wav,
                       tr.sigma.as<double>() + (int64_t)t.slot * tr.n_orb * tr.n_wav);
    PROM_HIP(hipGetLastError());
  }
  PROM_HIP(hipEventRecord(ev[2], s));
  // 3. fused tau kernel
  dim3 g((unsigned)((tr.n_wav + kBlock - 1) / kBlock), tr.n_orb);
  const double* sig = tr.sigma.as<double>();
  const double* recs = tr.recs.as<double>();
  const int32_t* counts = tr.counts.as<int32_t>();
  const double* ts = tr.tsum.as<double>();
  const double* fs = tr.fsum.as<double>();
  double* R = tr.R.as<double>();
  switch (tr.n_atoms) {
    case 1: hipLaunchKernelGGL(k_tau<1>, g, dim3(kBlock), 0, s, sig, recs, counts, ts, fs, 1, tr.n_pr, tr.n_orb, tr.n_wav, R); break;
    case 2: hipLaunchKernelGGL(k_tau<2>, g, dim3(kBlock), 0, s, sig, recs, counts, ts, fs, 2, tr.n_pr, tr.n_orb, tr.n_wav, R); break;
    case 3: hipLaunchKernelGGL(k_tau<3>, g, dim3(kBlock), 0, s, sig, recs, counts, ts, fs, 3, tr.n_pr, tr.n_orb, tr.n_wav, R); break;
    case 4: hipLaunchKernelGGL(k_tau<4>, g, dim3(kBlock), 0, s, sig, recs, counts, ts, fs, 4, tr.n_pr, tr.n_orb, tr.n_wav, R); break;
    default:
      hipLaunchKernelGGL(k_tau<0>, g, dim3(kBlock), (size_t)tr.n_atoms * kBlock * sizeof(double), s, sig, recs,
                         counts, ts, fs, tr.n_atoms, tr.n_pr, tr.n_orb, tr.n_wav, R);
  }
  PROM_HIP(hipGetLastError());
  *variant = tr.n_atoms <= 4 ? tr.n_atoms : 0;
  PROM_HIP(hipEventRecord(ev[3], s));
}

}  // namespace prom
