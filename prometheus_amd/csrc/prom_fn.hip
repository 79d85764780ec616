// Function-level kernels: n_interp_log / getSigmaAbs (gasProperties.py:34-51, :727-735), the Voigt
// tables (:672-715), density plugins (:143-516), the molecular lookup (:789-818), reductions and the
// light-curve band statistics (mainRetrieval.py:76-93).
#include "prom_device.h"

namespace prom {

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

// ------------------------------------------------------------------ molecular lookup (rgi_bracket, mol_value: prom_device.h)
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

// ------------------------------------------------------------------ gridded density (SERPENS)
__global__ void k_gridded(const double* __restrict__ g, int32_t nx, int32_t ny, int32_t nz, int64_t n,
                          const double* __restrict__ px, const double* __restrict__ py,
                          const double* __restrict__ pz, double* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  if (i >= n) return;
  out[i] = grid_value(g, nx, ny, nz, px[i], py[i], pz[i]);
}

void launch_gridded(hipStream_t s, const double* g, int32_t nx, int32_t ny, int32_t nz, int64_t n,
                    const double* px, const double* py, const double* pz, double* out) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gridded, dim3(grid_for(n, kBlock, (int64_t)1 << 31)), dim3(kBlock), 0, s, g, nx, ny, nz,
                     n, px, py, pz, out);
  PROM_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ interval records
// rec[i] = {x_i, E_i = 10^y_i, L_i = ln10 slope_i, x_{i+1}} with numpy.interp's slope of [x_i, x_{i+1}] (the
// same IEEE division as sigma_of's): on [x_i, x_{i+1}) numpy's 10^(y_i + slope_i (t - x_i)) is E_i e^a with
// a = L_i (t - x_i), which the polynomial sigma rows evaluate (k_sigma_poly).  The last node has L = 0 and
// x_{i+1} = +inf.  amax[i] = |L_i| (x_{i+1} - x_i), the largest |a| on the interval (0 for an empty one;
// NaN when y_i or y_{i+1} is not finite, which keeps such tables on the exp10 path).
__global__ void k_table_recs(const double* __restrict__ x, const double* __restrict__ y, int64_t n,
                             double4* __restrict__ rec, double* __restrict__ amax) {
  const int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  if (i >= n) return;
  const double xv = x[i], yv = y[i];
  double sl = 0.0, xn = __builtin_inf(), am = 0.0;
  if (i + 1 < n) {
    xn = x[i + 1];
    const double yn = y[i + 1];
    if (xn > xv) {
      sl = (yn - yv) / (xn - xv);
      am = fabs(sl * 2.302585092994046) * (xn - xv);
    }
    if (!__builtin_isfinite(yv) || !__builtin_isfinite(yn)) am = __builtin_nan("");
  } else if (!__builtin_isfinite(yv)) {
    am = __builtin_nan("");
  }
  rec[i] = make_double4(xv, exp10(yv), sl * 2.302585092994046, xn);
  if (amax) amax[i] = am;
}

// prom_transit_set's small inputs arrive in one DMA (descriptors + data, prom_api.hip Stager); a workgroup
// per descriptor scatters its bytes to the destination buffer (8-byte words, then the byte tail)
__global__ void __launch_bounds__(kBlock) k_scatter(const char* __restrict__ base, const ScatterDesc* __restrict__ d) {
  const ScatterDesc e = d[blockIdx.x];
  const char* src = base + e.src_off;
  char* dst = static_cast<char*>(e.dst);
  const int64_t words = e.bytes >> 3;
  if ((reinterpret_cast<uintptr_t>(dst) & 7) == 0) {
    for (int64_t i = threadIdx.x; i < words; i += kBlock)
      reinterpret_cast<uint64_t*>(dst)[i] = reinterpret_cast<const uint64_t*>(src)[i];
    for (int64_t i = (words << 3) + threadIdx.x; i < e.bytes; i += kBlock) dst[i] = src[i];
  } else {
    for (int64_t i = threadIdx.x; i < e.bytes; i += kBlock) dst[i] = src[i];
  }
}

void launch_scatter(hipStream_t s, const char* base, const ScatterDesc* d, int32_t n) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_scatter, dim3((unsigned)n), dim3(kBlock), 0, s, base, d);
  PROM_HIP(hipGetLastError());
}

void launch_table_recs(hipStream_t s, const double* x, const double* y, int64_t n, double4* rec, double* amax) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_table_recs, dim3(grid_for(n, kBlock, (int64_t)1 << 31)), dim3(kBlock), 0, s, x, y, n, rec,
                     amax);
  PROM_HIP(hipGetLastError());
}

// ------------------------------------------------------------------ reductions
__global__ void k_max(const double* __restrict__ v, int64_t n, double* __restrict__ out) {
  __shared__ double sm[kBlock];
  double m = -INFINITY;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
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
  if (threadIdx.x == 0) out[blockIdx.x] = sm[0];
}

// max (NaN-propagating) of a device array; scratch_dev must hold 1024 doubles
double reduce_max(hipStream_t s, const double* v, int64_t n, double* scratch_dev) {
  const unsigned g = grid_for(n, kBlock, 1024);
  hipLaunchKernelGGL(k_max, dim3(g), dim3(kBlock), 0, s, v, n, scratch_dev);
  PROM_HIP(hipGetLastError());
  std::vector<double> h(g);
  PROM_HIP(hipMemcpyAsync(h.data(), scratch_dev, sizeof(double) * g, hipMemcpyDeviceToHost, s));
  PROM_HIP(hipStreamSynchronize(s));
  double m = -INFINITY;
  for (double a : h) m = (a > m || a != a) ? a : m;
  return m;
}


// ---- light-curve band statistics (mainRetrieval.py:76-93) -------------------------------------------
// One workgroup per phase: strided partial sums / counts / maxima, then a fixed-order LDS tree, so the
// result does not depend on scheduling.  The max propagates NaN (numpy.max).
__global__ void __launch_bounds__(kBlock) k_band_stats(const double* __restrict__ R, const double* __restrict__ wav,
                                                       int64_t n_wav, int32_t n_bands,
                                                       const double* __restrict__ bounds, double* __restrict__ sum,
                                                       int64_t* __restrict__ count, double* __restrict__ mx) {
  __shared__ double ss[kBlock], sm[kBlock];
  __shared__ int64_t sc[kBlock];
  const int32_t o = blockIdx.x;
  const double* b = bounds + (int64_t)o * n_bands * 2;
  const double* r = R + (int64_t)o * n_wav;
  double acc = 0.0, m = -__builtin_inf();
  int64_t cnt = 0;
  for (int64_t w = threadIdx.x; w < n_wav; w += kBlock) {
    const double v = r[w], l = wav[w];
    m = (v > m || v != v || m != m) ? (m != m ? m : v) : m;
    bool sel = false;
    for (int32_t k = 0; k < n_bands; ++k) sel = sel || (l >= b[2 * k] && l <= b[2 * k + 1]);
    if (sel) {
      acc += v;
      ++cnt;
    }
  }
  ss[threadIdx.x] = acc;
  sm[threadIdx.x] = m;
  sc[threadIdx.x] = cnt;
  __syncthreads();
  for (int h = kBlock / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      ss[threadIdx.x] += ss[threadIdx.x + h];
      sc[threadIdx.x] += sc[threadIdx.x + h];
      const double a = sm[threadIdx.x], c = sm[threadIdx.x + h];
      sm[threadIdx.x] = (a != a || c != c) ? __builtin_nan("") : (c > a ? c : a);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    sum[o] = ss[0];
    count[o] = sc[0];
    mx[o] = sm[0];
  }
}

void launch_band_stats(hipStream_t s, const double* R, const double* wav, int32_t n_orb, int64_t n_wav,
                       int32_t n_bands, const double* bounds, double* sum, int64_t* count, double* mx) {
  hipLaunchKernelGGL(k_band_stats, dim3(n_orb), dim3(kBlock), 0, s, R, wav, n_wav, n_bands, bounds, sum, count, mx);
  PROM_HIP(hipGetLastError());
}

// Star.getFstarIntegrated, rotating branch (celestialBodies.py:299-311): per wavelength, the disk cells in
// the reference's loop order (phi outer, rho inner) accumulated one after the other,
//   acc += (((F * clv_c) * dphi) * drho) * rho_c,   F = 10^interp(lambda / shift_c)  (calculateRM :226-240),
// with the products rounded where numpy rounds them (-ffp-contract=off).  Four cells' lookups go out
// together (independent directory + window loads); the sum stays sequential.
__global__ void __launch_bounds__(kBlock) k_star_disk(const SigTabDev tb, const double* __restrict__ shift,
                                                       const double* __restrict__ clv, const double* __restrict__ rho,
                                                       int32_t n_cells, double dphi, double drho,
                                                       const double* __restrict__ wav, int64_t n_wav,
                                                       double* __restrict__ out) {
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < n_wav; w += (int64_t)gridDim.x * blockDim.x) {
    const double lam = wav[w];
    double acc = 0.0;
    int32_t c = 0;
    for (; c + 4 <= n_cells; c += 4) {
      double F[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) F[k] = sigma_of(lam / shift[c + k], tb);
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = acc + (((F[k] * clv[c + k]) * dphi) * drho) * rho[c + k];
    }
    for (; c < n_cells; ++c) acc = acc + (((sigma_of(lam / shift[c], tb) * clv[c]) * dphi) * drho) * rho[c];
    out[w] = acc;
  }
}

void launch_star_disk(hipStream_t s, const SigTabDev& tb, const double* shift, const double* clv, const double* rho,
                      int32_t n_cells, double dphi, double drho, const double* wav, int64_t n_wav, double* out) {
  if (n_wav == 0) return;
  hipLaunchKernelGGL(k_star_disk, dim3(grid_for(n_wav)), dim3(kBlock), 0, s, tb, shift, clv, rho, n_cells, dphi,
                     drho, wav, n_wav, out);
  PROM_HIP(hipGetLastError());
}

}  // namespace prom
