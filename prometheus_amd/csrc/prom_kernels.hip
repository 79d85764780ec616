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
//     k_tau<NS>   per (phase, wavelength): sigma_s = 10^interp(shift_o * lambda_w) - offset for each
//                 species, then tau over the active chords, exp(-tau), disk sum, ratio
#include "exp2_table.h"
#include "faddeeva.h"
#include "prom_internal.h"

namespace prom {

constexpr int kBlock = 256;

__constant__ double kExp2TableDev[PROM_EXP2_TABLE_N] = {
#define PROM_EXP2_TABLE_BODY
#include "exp2_table_body.h"
};

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

// One workgroup per phase.  Pass 1: F_out sum, transparent sum and the counts.  Pass 2: stream
// compaction of the active chords in chord order into packed records
//   {F_out / F_out_sum, N_0, .., N_{S-1}}
// (so R = sum_active w_c exp(-tau_c) + transparent fraction), their chord positions, and a flag
// for non-finite column densities (the tau kernel then takes the exact ocml path for that phase).
// counts[o] = {active, transparent, blocked, nonfinite, records}; tfrac[o] = transparent sum / F_out sum.
__global__ void __launch_bounds__(kBlock) k_compact(const int32_t* __restrict__ flags,
                                                    const double* __restrict__ fout,
                                                    const double* __restrict__ ncol, int32_t n_atoms,
                                                    int32_t n_pr, int32_t n_orb,
                                                    double* __restrict__ recs,
                                                    int32_t* __restrict__ act_ip,
                                                    int32_t* __restrict__ counts,
                                                    double* __restrict__ tfrac,
                                                    double* __restrict__ fsum) {
  const int32_t o = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __shared__ int32_t wcount[kBlock / 64];
  __shared__ double red[2][kBlock];
  __shared__ int32_t cnt[3][kBlock];
  int32_t ntr = 0, nbl = 0, nnf = 0;
  double tpart = 0.0, fpart = 0.0;
  for (int32_t ip = threadIdx.x; ip < n_pr; ip += kBlock) {
    const int32_t f = flags[(int64_t)o * n_pr + ip];
    const double fo = fout[ip];
    fpart += fo;
    if (f == 1) { tpart += fo; ++ntr; }
    if (f == 2) ++nbl;
    if (f == 0)
      for (int32_t s = 0; s < n_atoms; ++s)
        if (!__builtin_isfinite(ncol[((int64_t)s * n_orb + o) * n_pr + ip])) { ++nnf; break; }
  }
  red[0][threadIdx.x] = tpart;
  red[1][threadIdx.x] = fpart;
  cnt[0][threadIdx.x] = ntr;
  cnt[1][threadIdx.x] = nbl;
  cnt[2][threadIdx.x] = nnf;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
      cnt[0][threadIdx.x] += cnt[0][threadIdx.x + s];
      cnt[1][threadIdx.x] += cnt[1][threadIdx.x + s];
      cnt[2][threadIdx.x] += cnt[2][threadIdx.x + s];
    }
    __syncthreads();
  }
  const double fs = red[1][0];
  const int32_t stride = 1 + n_atoms;
  int32_t base = 0;
  for (int32_t chunk = 0; chunk < n_pr; chunk += kBlock) {
    const int32_t ip = chunk + threadIdx.x;
    const bool act = ip < n_pr && flags[(int64_t)o * n_pr + ip] == 0;
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
      r[0] = fout[ip] / fs;
      for (int32_t s = 0; s < n_atoms; ++s) r[1 + s] = ncol[((int64_t)s * n_orb + o) * n_pr + ip];
    }
    base += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    tfrac[o] = red[0][0] / fs;
    fsum[o] = fs;
    counts[o * 5 + 0] = base;
    counts[o * 5 + 1] = cnt[0][0];
    counts[o * 5 + 2] = cnt[1][0];
    counts[o * 5 + 3] = cnt[2][0];
    counts[o * 5 + 4] = base;   // records the tau kernel integrates (k_merge may lower it)
  }
}

// ---- chord merging ----------------------------------------------------------------------------
// Active chords of one phase whose column densities agree to 2^-40 relative in every species are
// integrated once with their summed weight.  Key of a chord: the IEEE bits of N_s shifted right by
// 12 (same key => same binade and |dN/N| < 2^-40).  For any merged chord, |tau' - tau| <= 2^-40 tau,
// so its term changes by at most w * 2^-40 * max_tau(tau e^-tau) = w * 2^-40 / e: the whole R moves
// by <= 3.4e-13.  Mirror-image chords (z -> -z about a body on the y axis, all built-in scenarios)
// merge pairwise; the central phase of a symmetric grid merges whole rings.
// One workgroup per phase; bitonic sort of (key_0, key_1, chord index) in LDS; phases with more
// than kMergeMax active chords, or non-finite columns, are left unmerged.
constexpr int kMergeBlock = 1024;
constexpr int kMergeMax = 4096;

__device__ __forceinline__ unsigned long long mkey(double v) {
  return __builtin_bit_cast(unsigned long long, v) >> 12;
}

__global__ void __launch_bounds__(kMergeBlock) k_merge(const double* __restrict__ recs, int32_t n_atoms,
                                                       int32_t n_pr, int32_t* __restrict__ counts,
                                                       double* __restrict__ mrecs) {
  __shared__ unsigned long long k0[kMergeMax];
  __shared__ unsigned long long k1[kMergeMax];
  __shared__ int32_t idx[kMergeMax];
  __shared__ int32_t gid[kMergeMax];
  __shared__ int32_t wsum[kMergeBlock / 64];
  const int32_t o = blockIdx.x;
  const int32_t n = counts[o * 5 + 0];
  const int32_t stride = 1 + n_atoms;
  const double* rec = recs + (int64_t)o * n_pr * stride;
  double* out = mrecs + (int64_t)o * n_pr * stride;
  if (n > kMergeMax || counts[o * 5 + 3] != 0 || n < 2) {
    for (int64_t i = threadIdx.x; i < (int64_t)n * stride; i += kMergeBlock) out[i] = rec[i];
    if (threadIdx.x == 0) counts[o * 5 + 4] = n;
    return;
  }
  int32_t P = 1;
  while (P < n) P <<= 1;
  for (int32_t i = threadIdx.x; i < P; i += kMergeBlock) {
    const bool v = i < n;
    k0[i] = v ? mkey(rec[(int64_t)i * stride + 1]) : ~0ull;
    k1[i] = (v && n_atoms > 1) ? mkey(rec[(int64_t)i * stride + 2]) : (v ? 0ull : ~0ull);
    idx[i] = v ? i : 0x7fffffff;
  }
  __syncthreads();
  for (int32_t size = 2; size <= P; size <<= 1) {
    for (int32_t stride_ = size >> 1; stride_ > 0; stride_ >>= 1) {
      for (int32_t t = threadIdx.x; t < P / 2; t += kMergeBlock) {
        const int32_t i = 2 * t - (t & (stride_ - 1));
        const int32_t j = i + stride_;
        const bool up = (i & size) == 0;
        const bool gt = (k0[i] > k0[j]) || (k0[i] == k0[j] && (k1[i] > k1[j] || (k1[i] == k1[j] && idx[i] > idx[j])));
        if (gt == up) {
          unsigned long long a = k0[i]; k0[i] = k0[j]; k0[j] = a;
          a = k1[i]; k1[i] = k1[j]; k1[j] = a;
          const int32_t b = idx[i]; idx[i] = idx[j]; idx[j] = b;
        }
      }
      __syncthreads();
    }
  }
  // group heads: first of a run of equal keys in every species
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int32_t base = 0;
  for (int32_t c0 = 0; c0 < n; c0 += kMergeBlock) {
    const int32_t i = c0 + threadIdx.x;
    bool head = false;
    if (i < n) {
      head = (i == 0) || k0[i] != k0[i - 1] || k1[i] != k1[i - 1];
      if (!head) {
        const double* a = rec + (int64_t)idx[i] * stride;
        const double* b = rec + (int64_t)idx[i - 1] * stride;
        for (int32_t s = 2; s < n_atoms && !head; ++s) head = mkey(a[1 + s]) != mkey(b[1 + s]);
      }
    }
    const unsigned long long m = __ballot(head);
    if (lane == 0) wsum[wid] = __popcll(m);
    __syncthreads();
    int32_t wb = 0, tot = 0;
    for (int w = 0; w < kMergeBlock / 64; ++w) {
      if (w < wid) wb += wsum[w];
      tot += wsum[w];
    }
    if (i < n) gid[i] = base + wb + __popcll(m & ((1ull << lane) - 1ull)) + (head ? 0 : -1);
    base += tot;
    __syncthreads();
  }
  // each head sums the weights of its run (sorted order) and writes the merged record
  for (int32_t i = threadIdx.x; i < n; i += kMergeBlock) {
    if (i > 0 && gid[i] == gid[i - 1]) continue;
    const double* a = rec + (int64_t)idx[i] * stride;
    double F = a[0];
    for (int32_t j = i + 1; j < n && gid[j] == gid[i]; ++j) F += rec[(int64_t)idx[j] * stride];
    double* r = out + (int64_t)gid[i] * stride;
    r[0] = F;
    for (int32_t s = 0; s < n_atoms; ++s) r[1 + s] = a[1 + s];
  }
  if (threadIdx.x == 0) counts[o * 5 + 4] = base;
}

// ---- fast exp: acc + F * 2^(y/2048) with a 2048-entry table in LDS --------------------------------
// y = -tau * 2048/ln2.  k = rint(y), d = y - k in [-1/2, 1/2],
//   2^(y/2048) = 2^(k >> 11) * T[k & 2047] * exp(d ln2/2048),
// exp(d c) = 1 + d (c + d (c^2/2 + d c^3/6)) with c = ln2/2048: truncation (c/2)^4/24 = 3.5e-17.
// Finite y only (non-finite column densities take the exact path); y below -2^31 saturates the
// integer conversion and ldexp flushes the term to 0, which is exp's own answer there.
constexpr double kExpC1 = 0.0003384507717577858;     // ln2 / 2048
constexpr double kExpC2 = 5.727446245172041e-08;     // c^2 / 2
constexpr double kExpC3 = 6.461528672932366e-12;     // c^3 / 6
constexpr double kMinus2048OverLn2 = -2954.639443740597;

__device__ __forceinline__ double acc_exp2k(double acc, double F, double y, const double* __restrict__ tab) {
  const double k = __builtin_rint(y);
  const int ki = (int)k;
  const double d = y - k;
  double t = __builtin_fma(d, kExpC3, kExpC2);
  t = __builtin_fma(d, t, kExpC1);
  const double e = __builtin_fma(d, t, 1.0);
  const double S = __builtin_amdgcn_ldexp(tab[ki & (PROM_EXP2_TABLE_N - 1)], ki >> 11);
  return __builtin_fma(F * S, e, acc);
}

// sigma of one atomic slot at (phase o, wavelength w): n_interp_log at shift_o * lambda_w.
__device__ __forceinline__ double slot_sigma(const SigTabDev& t, int32_t o, double lam) {
  return exp10(np_interp(t.shift[o] * lam, t.x, t.y, t.n)) - t.offset;
}

__device__ __forceinline__ void fill_exp_table(double* etab) {
  for (int i = threadIdx.x; i < PROM_EXP2_TABLE_N; i += kBlock) etab[i] = kExp2TableDev[i];
}

// Fused sigma lookup -> tau -> exp(-tau) -> disk sum -> ratio.  One thread per (phase o,
// wavelength w); the chord loop is uniform across the workgroup (all threads share the phase), so
// the packed chord records {lF, N_0..N_{S-1}} are read with scalar loads.
// NS: number of atomic slots (0 = runtime count, per-thread sigma in LDS).
// EXPK 1: table exp (exact ocml path for phases flagged non-finite);  0: ocml exp everywhere.
template <int NS, int EXPK>
__global__ void __launch_bounds__(kBlock) k_tau(const SigTabDev* __restrict__ tabs,
                                                const double* __restrict__ wav,
                                                const double* __restrict__ recs,
                                                const double* __restrict__ mrecs,
                                                const int32_t* __restrict__ act_ip,
                                                const double* __restrict__ fout,
                                                const int32_t* __restrict__ counts,
                                                const double* __restrict__ tfrac,
                                                const double* __restrict__ fsum, int32_t n_atoms_rt,
                                                int32_t n_pr, int64_t n_wav, double* __restrict__ R) {
  extern __shared__ double lds[];   // [2048] exp table | NS == 0: [n_atoms][kBlock] sigma
  double* etab = lds;
  double* sgl = lds + (EXPK ? PROM_EXP2_TABLE_N : 0);
  if (EXPK) fill_exp_table(etab);
  const int32_t o = blockIdx.y;
  const int64_t w = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  const bool live = w < n_wav;
  const double lam = wav[live ? w : n_wav - 1];
  const bool exact = !EXPK || counts[o * 5 + 3] != 0;
  const int32_t n_act = counts[o * 5 + (exact ? 0 : 4)];
  const int32_t ns = NS > 0 ? NS : n_atoms_rt;
  const int32_t stride = 1 + ns;
  const double* __restrict__ rec = (exact ? recs : mrecs) + (int64_t)o * n_pr * stride;
  const double scale = exact ? 1.0 : kMinus2048OverLn2;
  double acc = 0.0;
  double sp[NS > 0 ? NS : 1];
  if constexpr (NS > 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s) sp[s] = slot_sigma(tabs[s], o, lam) * scale;
  } else {
    for (int32_t s = 0; s < ns; ++s) sgl[s * kBlock + threadIdx.x] = slot_sigma(tabs[s], o, lam) * scale;
  }
  __syncthreads();
  if (!exact) {
    for (int32_t i = 0; i < n_act; ++i) {
      const double* r = rec + (int64_t)i * stride;
      double y;
      if constexpr (NS > 0) {
        y = r[1] * sp[0];
#pragma unroll
        for (int s = 1; s < NS; ++s) y = __builtin_fma(r[1 + s], sp[s], y);
      } else {
        y = r[1] * sgl[threadIdx.x];
        for (int32_t s = 1; s < ns; ++s) y = __builtin_fma(r[1 + s], sgl[s * kBlock + threadIdx.x], y);
      }
      acc = acc_exp2k(acc, r[0], y, etab);
    }
    if (live) R[(int64_t)o * n_wav + w] = acc + tfrac[o];
  } else {
    // exact path: tau in the reference's order (products then sums), ocml exp, F_out weights
    const int32_t* ipl = act_ip + (int64_t)o * n_pr;
    for (int32_t i = 0; i < n_act; ++i) {
      const double* r = rec + (int64_t)i * stride;
      double tau;
      if constexpr (NS > 0) {
        tau = r[1] * sp[0];
#pragma unroll
        for (int s = 1; s < NS; ++s) tau = tau + r[1 + s] * sp[s];
      } else {
        tau = r[1] * sgl[threadIdx.x];
        for (int32_t s = 1; s < ns; ++s) tau = tau + r[1 + s] * sgl[s * kBlock + threadIdx.x];
      }
      acc = acc + fout[ipl[i]] * exp(-tau);
    }
    if (live) R[(int64_t)o * n_wav + w] = (acc + tfrac[o] * fsum[o]) / fsum[o];
    (void)rec;
  }
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
  if (tr.merge && tr.exp_mode) {
    hipLaunchKernelGGL(k_merge, dim3(tr.n_orb), dim3(kMergeBlock), 0, s, tr.recs.as<double>(), tr.n_atoms,
                       tr.n_pr, tr.counts.as<int32_t>(), tr.mrecs.as<double>());
    PROM_HIP(hipGetLastError());
  }
  PROM_HIP(hipEventRecord(ev[1], s));
  // 2. (sigma is fused into the tau kernel; the event pair brackets nothing since round 1.2)
  PROM_HIP(hipEventRecord(ev[2], s));
  // 3. fused sigma -> tau -> exp -> disk-sum kernel
  dim3 g((unsigned)((tr.n_wav + kBlock - 1) / kBlock), tr.n_orb);
  const SigTabDev* tabs = tr.sigtab.as<SigTabDev>();
  const double* wav = tr.wav.as<double>();
  const double* recs = tr.recs.as<double>();
  const double* mrecs = (tr.merge && tr.exp_mode) ? tr.mrecs.as<double>() : recs;
  const int32_t* aip = tr.act_ip.as<int32_t>();
  const double* fo = tr.cfout.as<double>();
  const int32_t* counts = tr.counts.as<int32_t>();
  const double* tf = tr.tsum.as<double>();
  const double* fs = tr.fsum.as<double>();
  double* R = tr.R.as<double>();
  const int na = tr.n_atoms;
#define PROM_TAU(NSV, EK)                                                                              \
  hipLaunchKernelGGL((k_tau<NSV, EK>), g, dim3(kBlock),                                                \
                     ((EK) ? PROM_EXP2_TABLE_N * sizeof(double) : 0) +                                  \
                         ((NSV) == 0 ? (size_t)na * kBlock * sizeof(double) : 0),                      \
                     s, tabs, wav, recs, mrecs, aip, fo, counts, tf, fs, na, tr.n_pr, tr.n_wav, R)
#define PROM_TAU_NS(EK)                 \
  switch (na) {                         \
    case 1: PROM_TAU(1, EK); break;     \
    case 2: PROM_TAU(2, EK); break;     \
    case 3: PROM_TAU(3, EK); break;     \
    case 4: PROM_TAU(4, EK); break;     \
    default: PROM_TAU(0, EK);           \
  }
  if (tr.exp_mode) { PROM_TAU_NS(1) } else { PROM_TAU_NS(0) }
#undef PROM_TAU_NS
#undef PROM_TAU
  PROM_HIP(hipGetLastError());
  *variant = (na <= 4 ? na : 0) + (tr.exp_mode ? 10 : 0);
  PROM_HIP(hipEventRecord(ev[3], s));
}

}  // namespace prom
