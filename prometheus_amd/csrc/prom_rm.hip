// Stellar-spectrum fused tau kernel (gasProperties.py:1180-1219: CLV + Rossiter-McLaughlin).
#include "prom_device.h"

namespace prom {

// ---- stellar spectrum path (gasProperties.py:1180-1219 with Fstar_function set) ----------------------
// F(c, w) = rho_c * (F_star(lambda_w / s_c) * clv_c) differs per chord AND wavelength (the Rossiter-
// McLaughlin shift s_c moves the stellar lines across the disk), so neither the flat-star F_out
// factorisation nor the windowed tail moments apply: every (chord, wavelength) flux is evaluated.
// One thread per wavelength, kRmP phases per workgroup.  F is computed once per (chord, wavelength)
// and shared by the workgroup's phases; chords transparent at every phase of the group add F to one
// shared sum (exp(-tau) == 1 to the last ulp), the others are resolved per phase from a bit mask.
// F_star(t) = 10^(f_k + slope_k (t - x_k)) is evaluated as 10^f_k * exp(ln10 slope_k (t - x_k)) on the
// LDS copy of the star-table slice that the workgroup's targets t = lambda / s can reach (prom_api.hip
// rm_slices), bracketed through a slice-local bucket directory; a tile whose slice exceeds kRmStarMax
// nodes uses the global lookup (sigma_of).  With one shift for every chord (no rotation) F_star is
// evaluated once per wavelength.
constexpr int kRmP = 8;            // phases per workgroup
constexpr int kRmChunk = 64;       // chords staged in LDS per sweep
constexpr int kRmGroup = 4;        // chords whose F_star lookups are interleaved
constexpr int kRmDir = 2 * kRmStarMax;   // slice-directory buckets (at most)
constexpr double kLn10 = 2.302585092994045684;

// exp(a) for the F_star interpolation factor (|a| <= ln10 |f_k+1 - f_k|): the 256-entry table scheme of
// acc_exp256 (relative error ~ |a| 2^-53 from the argument scaling)
__device__ __forceinline__ double exp_tab(double a, const double* __restrict__ tab) {
  const double y = a * -kM256Ln2;
  const double k = __builtin_rint(y);
  const int ki = (int)k;
  const double d = y - k;
  double p = __builtin_fma(d, kE256C5, kE256C4);
  p = __builtin_fma(d, p, kE256C3);
  p = __builtin_fma(d, p, kE256C2);
  p = __builtin_fma(d, p, kE256C1);
  p = __builtin_fma(d, p, 1.0);
  return __builtin_amdgcn_ldexp(tab[ki & 255], ki >> 8) * p;
}

template <int NSMAX, bool OCML, bool UNISTAR>
__global__ void __launch_bounds__(kBlock) k_tau_rm(const SigTabDev* __restrict__ tabs, int32_t na,
                                                   const SigTabDev star, const int32_t* __restrict__ slices,
                                                   const double* __restrict__ wav, int64_t n_wav,
                                                   const double* __restrict__ crho,
                                                   const double* __restrict__ cclv,
                                                   const double* __restrict__ cshift,
                                                   const int32_t* __restrict__ flags,
                                                   const double* __restrict__ ncol, int32_t n_pr,
                                                   int32_t n_orb, int32_t* __restrict__ counts,
                                                   double* __restrict__ R) {
  __shared__ double sexp[256];
  __shared__ double sx[kRmStarMax], sF[kRmStarMax], sc[kRmStarMax];
  __shared__ int16_t sdir[kRmDir];
  __shared__ double sRho[kRmChunk], sClv[kRmChunk], sSh[kRmChunk];
  __shared__ double sN[kRmP * NSMAX * kRmChunk];
  __shared__ int32_t sMask[kRmChunk];
  __shared__ int32_t scnt[kRmP * 3];
  sexp[threadIdx.x] = kExp2TableDev[8 * threadIdx.x];   // kBlock == 256
  const int32_t o0 = blockIdx.y * kRmP;
  const int32_t np = n_orb - o0 < kRmP ? n_orb - o0 : kRmP;
  const int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool live = w < n_wav;
  const double lam = wav[live ? w : n_wav - 1];
  // chord counts per phase (stats), by the first workgroup of each phase group
  if (blockIdx.x == 0 && counts) {
    if (threadIdx.x < kRmP * 3) scnt[threadIdx.x] = 0;
    __syncthreads();
    for (int p = 0; p < np; ++p)
      for (int32_t i = threadIdx.x; i < n_pr; i += kBlock) {
        const int32_t f = flags[(int64_t)(o0 + p) * n_pr + i];
        atomicAdd(&scnt[p * 3 + (f < 0 ? 0 : (f > 2 ? 2 : f))], 1);
      }
    __syncthreads();
    if (threadIdx.x < np) {
      int32_t* cp = counts + (int64_t)(o0 + threadIdx.x) * kCnt;
      cp[0] = scnt[threadIdx.x * 3];
      cp[1] = scnt[threadIdx.x * 3 + 1];
      cp[2] = scnt[threadIdx.x * 3 + 2];
      for (int k = 3; k < kCnt; ++k) cp[k] = 0;
    }
  }
  // star-table slice {lo, m, half}: nodes lo .. lo+m-1 as (x_k, 10^f_k, ln10 slope_k) + a directory of
  // nb = 4 half buckets over [x_0, x_m-1]: sdir[j] = last node <= x_0 + j h
  const int32_t* sl = slices + 3 * (int64_t)blockIdx.x;
  const int64_t lo = sl[0];
  const int32_t m = UNISTAR ? 0 : sl[1], half = sl[2];
  const int32_t nb = 4 * half < kRmDir ? 4 * half : kRmDir;
  double sx0 = 0.0, inv_h = 0.0;
  if (m > 0) {
    for (int i = threadIdx.x; i < m; i += kBlock) {
      const double x0 = star.x[lo + i], f0 = star.y[lo + i];
      sx[i] = x0;
      sF[i] = exp10(f0);                       // star tables have offset 0 (prom_transit_set)
      sc[i] = i + 1 < m ? ((star.y[lo + i + 1] - f0) / (star.x[lo + i + 1] - x0)) * kLn10 : 0.0;
    }
    sx0 = star.x[lo];
    const double span = star.x[lo + m - 1] - sx0;
    inv_h = span > 0.0 ? (double)nb / span : 0.0;
    __syncthreads();
    for (int j = threadIdx.x; j < nb; j += kBlock) {
      const double b = sx0 + (double)j * (span / (double)nb);
      int pos = 0;
      for (int st = half; st > 0; st >>= 1) pos += (pos + st < m && sx[pos + st] <= b) ? st : 0;
      sdir[j] = (int16_t)pos;
    }
  }
  // sigma_s at each of this thread's phases (shift_o * lambda, as getLOSopticalDepth_Batch)
  double sg[kRmP][NSMAX];
#pragma unroll
  for (int p = 0; p < kRmP; ++p)
#pragma unroll
    for (int s = 0; s < NSMAX; ++s)
      sg[p][s] = (p < np && s < na) ? sigma_of(tabs[s].shift[o0 + p] * lam, tabs[s]) : 0.0;
  double fstar_uni = 0.0;
  if constexpr (UNISTAR) fstar_uni = sigma_of(lam / cshift[0], star);
  double in[kRmP];
#pragma unroll
  for (int p = 0; p < kRmP; ++p) in[p] = 0.0;
  double out = 0.0, tall = 0.0;
  for (int32_t c0 = 0; c0 < n_pr; c0 += kRmChunk) {
    const int nch = n_pr - c0 < kRmChunk ? n_pr - c0 : kRmChunk;
    __syncthreads();
    for (int i = threadIdx.x; i < nch; i += kBlock) {
      sRho[i] = crho[c0 + i];
      sClv[i] = cclv[c0 + i];
      sSh[i] = cshift[c0 + i];
      int32_t am = 0, bm = 0;
      for (int p = 0; p < np; ++p) {
        const int32_t f = flags[(int64_t)(o0 + p) * n_pr + c0 + i];
        am |= (f == 0) << p;
        bm |= (f == 2) << p;
      }
      sMask[i] = am | (bm << 8);
    }
    for (int i = threadIdx.x; i < na * np * nch; i += kBlock) {
      const int sp = i / nch, c = i - sp * nch;     // sp = s * np + p
      const int s = sp / np, p = sp - s * np;
      sN[(p * NSMAX + s) * kRmChunk + c] = ncol[((int64_t)s * n_orb + o0 + p) * n_pr + c0 + c];
    }
    __syncthreads();
    for (int cg = 0; cg < nch; cg += kRmGroup) {
      // F_star for kRmGroup chords at once: their LDS chains (directory -> bracket steps -> node ->
      // table exp) are independent, so interleaving them hides the LDS latency
      double fsg[kRmGroup];
      if constexpr (UNISTAR) {
#pragma unroll
        for (int u = 0; u < kRmGroup; ++u) fsg[u] = fstar_uni;
      } else if (m > 0) {
        double t[kRmGroup];
        int k[kRmGroup];
#pragma unroll
        for (int u = 0; u < kRmGroup; ++u) {
          t[u] = lam / sSh[cg + u < nch ? cg + u : nch - 1];
          const double fj = (t[u] - sx0) * inv_h;
          const int j = !(fj >= 1.0) ? 1 : (fj >= (double)nb ? nb : (int)fj);
          k[u] = sdir[j - 1];
        }
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int u = 0; u < kRmGroup; ++u) k[u] += (k[u] + 1 < m && sx[k[u] + 1] <= t[u]) ? 1 : 0;
        const double xlast = sx[m - 1];
#pragma unroll
        for (int u = 0; u < kRmGroup; ++u) {
          const double tu = t[u];
          if (!(tu >= sx0) || tu >= xlast) {
            // below the table (the slice starts at node 0) / at or beyond the table's last node
            fsg[u] = tu != tu ? tu : (tu >= xlast ? sF[m - 1] : sF[0]);
            continue;
          }
          int kk = k[u];
          if (sx[kk + 1] <= tu) {                      // crowded bucket: bisect the rest of the slice
            int a = kk + 1, b = m - 1;                 // sx[a] <= t < sx[b]
            while (b - a > 1) {
              const int mid = (a + b) >> 1;
              if (sx[mid] <= tu) a = mid; else b = mid;
            }
            kk = a;
          }
          const double xk = sx[kk];
          const double arg = sc[kk] * (tu - xk);
          if (xk == tu) fsg[u] = sF[kk];
          else if (__builtin_isfinite(arg)) fsg[u] = sF[kk] * exp_tab(arg, sexp);
          else fsg[u] = sigma_of(tu, star);          // infinite slope (repeated node): np.interp's rules
        }
      } else {
#pragma unroll
        for (int u = 0; u < kRmGroup; ++u) fsg[u] = sigma_of(lam / sSh[cg + u < nch ? cg + u : nch - 1], star);
      }
#pragma unroll
      for (int u = 0; u < kRmGroup; ++u) {
        const int c = cg + u;
        if (c >= nch) break;
        const double fs = fsg[u];
        const double Fc = sRho[c] * (fs * sClv[c]);
        out += Fc;
        const int32_t mk = __builtin_amdgcn_readfirstlane(sMask[c]);
        if (mk == 0) {
          tall += Fc;                                  // transparent at every phase of the group
          continue;
        }
#pragma unroll
        for (int p = 0; p < kRmP; ++p) {
          if (p >= np) break;
          if ((mk >> p) & 1) {
            double tau = 0.0;
#pragma unroll
            for (int s = 0; s < NSMAX; ++s)
              if (s < na) tau += sN[(p * NSMAX + s) * kRmChunk + c] * sg[p][s];
            if (OCML || !(tau < 700.0 && tau > -700.0)) in[p] += Fc * exp(-tau);
            else in[p] = acc_exp256(in[p], Fc, tau * kM256Ln2, sexp);
          } else if (!((mk >> (p + 8)) & 1)) {
            in[p] += Fc;                               // transparent at this phase
          }
        }
      }
    }
  }
  if (live) {
#pragma unroll
    for (int p = 0; p < kRmP; ++p)
      if (p < np) R[(int64_t)(o0 + p) * n_wav + w] = (in[p] + tall) / out;
  }
}

void launch_tau_rm(hipStream_t s, TransitDev& tr, RunSlot& rs, int32_t na, hipEvent_t* ev) {
    const SigTabDev star = tr.star_tab;
    const dim3 g((unsigned)((tr.n_wav + kBlock - 1) / kBlock), (unsigned)((tr.n_orb + kRmP - 1) / kRmP));
#define PROM_RM(NSV, OC)                                                                                \
  do {                                                                                                  \
    if (tr.star_uniform) { PROM_RM2(NSV, OC, true); } else { PROM_RM2(NSV, OC, false); }                 \
  } while (0)
#define PROM_RM2(NSV, OC, UV)                                                                           \
  hipExtLaunchKernelGGL((k_tau_rm<NSV, OC, UV>), g, dim3(kBlock), 0, s, ev ? ev[2] : nullptr, ev ? ev[3] : nullptr, 0, \
                        tr.sigtab.as<SigTabDev>(), na, star, tr.rm_slices.as<int32_t>(), tr.wav.as<double>(), \
                        tr.n_wav, tr.crho.as<double>(), tr.cclv.as<double>(), tr.cshift.as<double>(),     \
                        rs.flags.as<int32_t>(), rs.ncol.as<double>(), tr.n_pr, tr.n_orb,                  \
                        tr.count_evals ? rs.counts.as<int32_t>() : nullptr, rs.R.as<double>())
#define PROM_RM_NS(OC)                       \
  if (na <= 1) PROM_RM(1, OC);               \
  else if (na == 2) PROM_RM(2, OC);          \
  else if (na <= 4) PROM_RM(4, OC);          \
  else PROM_RM(8, OC);
    PROM_REQUIRE(tr.n_mol == 0 && na <= 8, "transit: the stellar-spectrum path takes <= 8 atomic constituents and no molecules");
    if (tr.exp_mode) { PROM_RM_NS(false) } else { PROM_RM_NS(true) }
#undef PROM_RM_NS
#undef PROM_RM
#undef PROM_RM2
}

}  // namespace prom
