// Doppler-shifted cross-section rows for the fast transit path (launched by launch_transit in
// prom_transit.hip when every phase has its own Doppler factor).
#include "prom_device.h"

namespace prom {

constexpr int kSigRowChunk = 8;   // rows kept in registers per pass over the species
static_assert(kSigBlockW == kBlock, "sigma segments are built per kBlock wavelengths");

// ---- Doppler-shifted cross-section rows (orbital Doppler shift: one row per phase) ----------------
// One workgroup per 256-wavelength block, a thread per wavelength, looping over the rows (phases).
// The host (prom_api.hip sigma segments) gives, per block and atomic slot, the table nodes
// [lo, lo + m) that every row's shifted targets shift_o * lambda_w fall between: positive factors
// and IEEE multiplication are monotone, so fl(shift_o lambda_w) lies in [fl(s_min lambda_first),
// fl(s_max lambda_last)].  Those nodes go to LDS once per 8 rows, with numpy.interp's slope of
// each interval divided once per node instead of once per target; a target's bracket is a
// bisection of the slice for a chunk's first row, then a short walk from the previous row's
// bracket (the rows' factors are close).  Blocks whose slice exceeds kSigSeg nodes (the
// high-resolution line windows, where the table is 10x finer than the grid) keep the per-target
// directory gather of sigma_of.  Same bracket rule, slope, products and exp10 as sigma_of /
// sigma_multi: the rows are bit-for-bit those of the per-target lookups.
static_assert(kSigBlockW == kBlock, "sigma segments are built per kBlock wavelengths");

template <int NSIG>
__global__ void __launch_bounds__(kBlock) k_sigma_rows(const SigTabs4 tabv, const double* __restrict__ wav, int64_t n_wav,
                                                 int32_t n_rows, const int2* __restrict__ seg,
                                                 double* __restrict__ sig, float4* __restrict__ tq, int32_t merge_sp,
                                                 double nscale_m, uint8_t* __restrict__ zfl) {
  __shared__ double sx[kSigSeg], sy[kSigSeg], ss[kSigSeg];
  const int64_t wb = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int64_t w = wb * kBlock + tid;
  const bool live = w < n_wav;
  const double lam = wav[live ? w : n_wav - 1];
  const int64_t n_halves = 2 * ((n_wav + kTW - 1) / kTW);
  const int64_t hw = wb * (kBlock / 64) + (tid >> 6);
  const int32_t nse = merge_sp ? 1 : NSIG;
  for (int32_t r0 = 0; r0 < n_rows; r0 += kSigRowChunk) {
    double Y[kSigRowChunk], Q[kSigRowChunk];
    uint32_t zbits = 0;
#pragma unroll
    for (int r = 0; r < kSigRowChunk; ++r) { Y[r] = 0.0; Q[r] = 0.0; }
#pragma unroll
    for (int s = 0; s < NSIG; ++s) {
      const SigTabDev& tb = tabv.t[s];
      const int2 sg = seg[wb * NSIG + s];
      const int32_t m = sg.y;
      __syncthreads();   // the previous species' slice is no longer read
      if (m > 0) {
        for (int32_t i = tid; i < m; i += kBlock) {
          const double xv = tb.x[sg.x + i], yv = tb.y[sg.x + i];
          sx[i] = xv;
          sy[i] = yv;
          if (i + 1 < m) {
            const double xn = tb.x[sg.x + i + 1], yn = tb.y[sg.x + i + 1];
            ss[i] = (yn - yv) / (xn - xv);
          }
        }
      }
      __syncthreads();
      const double f_first = tb.y[0], f_last = tb.y[tb.n - 1];
      int32_t k = 0;
      if (m > 0) {   // the chunk's first row: bisection, sx[a] <= t < sx[b] (out-of-range t: an end)
        const double t = tb.shift[r0] * lam;
        int32_t a = 0, b = m - 1;
        while (b - a > 1) {
          const int32_t mid = (a + b) >> 1;
          if (sx[mid] <= t) a = mid; else b = mid;
        }
        k = a;
      }
#pragma unroll
      for (int r = 0; r < kSigRowChunk; ++r) {
        const int32_t orow = r0 + r;
        if (orow >= n_rows) break;
        const double t = tb.shift[orow] * lam;
        double v;
        if (m > 0) {
          double rv;
          if (t != t) rv = t;
          else if (!(t >= tb.xfirst)) rv = f_first;
          else if (t >= tb.xlast) rv = f_last;
          else {
            // walk from the previous row's bracket (the rows' factors are close)
            while (k > 0 && sx[k] > t) --k;
            while (k < m - 2 && sx[k + 1] <= t) ++k;
            const double xa = sx[k], fa = sy[k];
            if (xa == t) rv = fa;
            else {
              const double slope = ss[k];
              rv = slope * (t - xa) + fa;
              if (rv != rv) {
                const double xb = sx[k + 1], fb = sy[k + 1];
                rv = slope * (t - xb) + fb;
                if (rv != rv && fa == fb) rv = fa;
              }
            }
          }
          v = exp10(rv) - tb.offset;
        } else {
          v = sigma_of(t, tb);
        }
        if (merge_sp) {
          const double cv = tb.chi * v;
          if (!(cv > 0.0)) zbits |= 1u << r;
          Y[r] += cv;
        } else {
          if (live) sig[((int64_t)orow * nse + s) * n_wav + w] = v;
          const double qs = v * tb.nscale;
          Q[r] += qs > 0.0 ? qs : 0.0;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kSigRowChunk; ++r) {
      const int32_t orow = r0 + r;
      if (orow >= n_rows) break;
      double Qv = Q[r];
      if (merge_sp) {
        if (live) {
          sig[(int64_t)orow * n_wav + w] = Y[r];
          zfl[(int64_t)orow * n_wav + w] = (zbits >> r) & 1u;
        }
        const double qs = Y[r] * nscale_m;
        Qv = qs > 0.0 ? qs : 0.0;
      }
      const float qf = (float)Qv;
      float qh = qf * (1.0f + 0x1p-20f), ql = qf * (1.0f - 0x1p-20f);
      for (int off = 32; off > 0; off >>= 1) {
        qh = fmaxf(qh, __shfl_xor(qh, off, 64));
        ql = fminf(ql, __shfl_xor(ql, off, 64));
      }
      const bool bad = __ballot(!(Qv <= 1.0e100)) != 0ull;
      if (lane == 0 && hw < n_halves)
        reinterpret_cast<float2*>(tq)[(int64_t)orow * n_halves + hw] =
            bad ? make_float2(-1.0f, 0.0f) : make_float2(ql, qh);
    }
  }
}


void launch_sigma_rows(hipStream_t s, int32_t nsig, const SigTabs4& tabv, const double* wav, int64_t n_wav,
                       int32_t n_rows, const int2* seg, double* sig, float4* tq, int32_t merge_sp, double nscale_m,
                       uint8_t* zfl, hipEvent_t ev_start) {
  const unsigned nb = grid_for(n_wav);
#define PROM_SIGR(NS)                                                                                        \
  hipExtLaunchKernelGGL((k_sigma_rows<NS>), dim3(nb), dim3(kBlock), 0, s, ev_start, nullptr, 0, tabv, wav, n_wav, \
                        n_rows, seg, sig, tq, merge_sp, nscale_m, zfl)
  switch (nsig) {
    case 1: PROM_SIGR(1); break;
    case 2: PROM_SIGR(2); break;
    case 3: PROM_SIGR(3); break;
    default: PROM_SIGR(4); break;
  }
#undef PROM_SIGR
  PROM_HIP(hipGetLastError());
}

}  // namespace prom
