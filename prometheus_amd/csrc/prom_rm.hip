// Stellar-spectrum fused tau kernel (gasProperties.py:1180-1219: CLV + Rossiter-McLaughlin).
#include "prom_device.h"

namespace prom {

// ---- stellar spectrum path (gasProperties.py:1180-1219 with Fstar_function set) ----------------------
// F(c, w) = rho_c * (F_star(lambda_w / s_c) * clv_c) differs per chord AND wavelength (the Rossiter-
// McLaughlin shift s_c moves the stellar lines across the disk), so neither the flat-star F_out
// factorisation nor the windowed tail moments apply: every (chord, wavelength) flux is evaluated.
// One thread per wavelength, RP phases per workgroup (2, launch_tau_rm).  The unocculted flux Fout(w) = sum_c F(c, w) is a
// per-set quantity (k_rm_fout); a run visits only the chords blocked or active at some phase of its group
// (F once per such (chord, wavelength), shared by the group's phases) and subtracts their loss from Fout.
// F_star(t) = 10^(f_k + slope_k (t - x_k)) is evaluated as 10^f_k * exp(ln10 slope_k (t - x_k)) on the
// LDS copy of the star-table slice that the workgroup's targets t = lambda / s can reach (prom_api.hip
// rm_slices), bracketed through a slice-local bucket directory; a tile whose slice exceeds kRmStarMax
// nodes uses the global lookup (sigma_of).  With one shift for every chord (no rotation) F_star is
// evaluated once per wavelength.
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

// F_star(lambda_w / s_c) for kRmGroup chords of the LDS list at once (their LDS chains -- directory, bracket steps,
// node, table exp -- are independent, so interleaving them hides the LDS latency)
struct RmStar {
  const double* sx;
  const double* sF;
  const double* sc;
  const int16_t* sdir;
  const double* sexp;
  double sx0, inv_h;
  int32_t m, nb;
};

template <bool UNISTAR>
__device__ __forceinline__ void rm_fstar(double (&fsg)[kRmGroup], double lam, const double (&sh)[kRmGroup],
                                         const RmStar& st, const SigTabDev& star, double fstar_uni) {
  if constexpr (UNISTAR) {
#pragma unroll
    for (int u = 0; u < kRmGroup; ++u) fsg[u] = fstar_uni;
  } else if (st.m > 0) {
    const int32_t m = st.m, nb = st.nb;
    double t[kRmGroup];
    int k[kRmGroup];
#pragma unroll
    for (int u = 0; u < kRmGroup; ++u) {
      t[u] = lam / sh[u];
      const double fj = (t[u] - st.sx0) * st.inv_h;
      const int j = !(fj >= 1.0) ? 1 : (fj >= (double)nb ? nb : (int)fj);
      k[u] = st.sdir[j - 1];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int u = 0; u < kRmGroup; ++u) k[u] += (k[u] + 1 < m && st.sx[k[u] + 1] <= t[u]) ? 1 : 0;
    const double xlast = st.sx[m - 1];
#pragma unroll
    for (int u = 0; u < kRmGroup; ++u) {
      const double tu = t[u];
      if (!(tu >= st.sx0) || tu >= xlast) {
        // below the table (the slice starts at node 0) / at or beyond the table's last node
        fsg[u] = tu != tu ? tu : (tu >= xlast ? st.sF[m - 1] : st.sF[0]);
        continue;
      }
      int kk = k[u];
      if (st.sx[kk + 1] <= tu) {                   // crowded bucket: bisect the rest of the slice
        int a = kk + 1, b = m - 1;                 // sx[a] <= t < sx[b]
        while (b - a > 1) {
          const int mid = (a + b) >> 1;
          if (st.sx[mid] <= tu) a = mid; else b = mid;
        }
        kk = a;
      }
      const double xk = st.sx[kk];
      const double arg = st.sc[kk] * (tu - xk);
      if (xk == tu) fsg[u] = st.sF[kk];
      else if (__builtin_isfinite(arg)) fsg[u] = st.sF[kk] * exp_tab(arg, st.sexp);
      else fsg[u] = sigma_of(tu, star);          // infinite slope (repeated node): np.interp's rules
    }
  } else {
#pragma unroll
    for (int u = 0; u < kRmGroup; ++u) fsg[u] = sigma_of(lam / sh[u], star);
  }
}

// Stages the workgroup's star-table slice {lo, m, half} in LDS: nodes lo .. lo+m-1 as (x_k, 10^f_k, ln10 slope_k)
// + a directory of nb = 4 half buckets over [x_0, x_m-1]: sdir[j] = last node <= x_0 + j h
template <bool UNISTAR>
__device__ __forceinline__ RmStar rm_stage(const SigTabDev& star, const int32_t* __restrict__ slices, double* sx,
                                           double* sF, double* sc, int16_t* sdir, const double* sexp) {
  RmStar st{sx, sF, sc, sdir, sexp, 0.0, 0.0, 0, 0};
  const int32_t* sl = slices + 3 * (int64_t)blockIdx.x;
  const int64_t lo = sl[0];
  const int32_t m = UNISTAR ? 0 : sl[1], half = sl[2];
  st.m = m;
  st.nb = 4 * half < kRmDir ? 4 * half : kRmDir;
  if (m > 0) {
    for (int i = threadIdx.x; i < m; i += kBlock) {
      const double x0 = star.x[lo + i], f0 = star.y[lo + i];
      sx[i] = x0;
      sF[i] = exp10(f0);                       // star tables have offset 0 (prom_transit_set)
      sc[i] = i + 1 < m ? ((star.y[lo + i + 1] - f0) / (star.x[lo + i + 1] - x0)) * kLn10 : 0.0;
    }
    st.sx0 = star.x[lo];
    const double span = star.x[lo + m - 1] - st.sx0;
    st.inv_h = span > 0.0 ? (double)st.nb / span : 0.0;
    __syncthreads();
    for (int j = threadIdx.x; j < st.nb; j += kBlock) {
      const double b = st.sx0 + (double)j * (span / (double)st.nb);
      int pos = 0;
      for (int stp = half; stp > 0; stp >>= 1) pos += (pos + stp < m && sx[pos + stp] <= b) ? stp : 0;
      sdir[j] = (int16_t)pos;
    }
  }
  return st;
}

// Per set: the unocculted flux Fout(w) = sum_c F(c, w) over every chord in chord order (gasProperties.py:1221-1245,
// the denominator of R), F(c, w) = rho_c (F_star(lambda_w / s_c) clv_c).  It depends only on the chord grid, the
// star's spectrum and rotation and the wavelengths -- none of which a run changes -- so runs reuse it.
template <bool UNISTAR>
__global__ void __launch_bounds__(kBlock) k_rm_fout(const SigTabDev star, const int32_t* __restrict__ slices,
                                                    const double* __restrict__ wav, int64_t n_wav,
                                                    const double* __restrict__ crho, const double* __restrict__ cclv,
                                                    const double* __restrict__ cshift, int32_t n_pr,
                                                    double* __restrict__ fo, double* __restrict__ ftab) {
  __shared__ double sexp[256];
  __shared__ double sx[kRmStarMax], sF[kRmStarMax], sc[kRmStarMax];
  __shared__ int16_t sdir[kRmDir];
  sexp[threadIdx.x] = kExp2TableDev[8 * threadIdx.x];   // kBlock == 256
  const int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const double lam = wav[w < n_wav ? w : n_wav - 1];
  const RmStar st = rm_stage<UNISTAR>(star, slices, sx, sF, sc, sdir, sexp);
  __syncthreads();
  double fstar_uni = 0.0;
  if constexpr (UNISTAR) fstar_uni = sigma_of(lam / cshift[0], star);
  double out = 0.0;
  for (int32_t c0 = 0; c0 < n_pr; c0 += kRmGroup) {
    double sh[kRmGroup], fsg[kRmGroup];
#pragma unroll
    for (int u = 0; u < kRmGroup; ++u) sh[u] = cshift[c0 + u < n_pr ? c0 + u : n_pr - 1];
    rm_fstar<UNISTAR>(fsg, lam, sh, st, star, fstar_uni);
#pragma unroll
    for (int u = 0; u < kRmGroup; ++u)
      if (c0 + u < n_pr) {
        const double F = crho[c0 + u] * (fsg[u] * cclv[c0 + u]);
        if (ftab && w < n_wav) ftab[(int64_t)(c0 + u) * n_wav + w] = F;   // (chord-major: a run reads rows)
        out += F;
      }
  }
  if (w < n_wav) fo[w] = out;
}

// Per run: R(o, w) = (Fout(w) - loss(o, w)) / Fout(w), loss = sum over the chords blocked at o of F + sum over the
// chords active at o of F (1 - e^-tau) -- the reference's sum_unblocked F e^-tau with every transparent chord's
// exact F (e^-tau == 1 to the last ulp) left inside Fout.  Only chords blocked or active at some phase of the
// workgroup's group are visited (a 64-chord chunk is compacted by ballot), so F_star is looked up for those alone.
// FT: F(c, w) read from the per-set table k_rm_fout wrote (ftab[c][w], the same value), no star-table lookups here.
template <int NSMAX, bool OCML, bool UNISTAR, bool FT, int RP>
__global__ void __launch_bounds__(kBlock) k_tau_rm(const SigTabDev* __restrict__ tabs, int32_t na,
                                                   const SigTabDev star, const int32_t* __restrict__ slices,
                                                   const double* __restrict__ wav, int64_t n_wav,
                                                   const double* __restrict__ crho,
                                                   const double* __restrict__ cclv,
                                                   const double* __restrict__ cshift,
                                                   const double* __restrict__ fout_w,
                                                   const int32_t* __restrict__ flags,
                                                   const double* __restrict__ ncol, int32_t n_pr,
                                                   int32_t n_orb, int32_t* __restrict__ counts,
                                                   const double* __restrict__ ftab, double* __restrict__ R) {
  __shared__ double sexp[256];
  constexpr int SM = FT ? 1 : kRmStarMax;
  __shared__ double sx[SM], sF[SM], sc[SM];
  __shared__ int16_t sdir[FT ? 1 : kRmDir];
  __shared__ double sRho[kRmChunk], sClv[kRmChunk], sSh[kRmChunk];
  __shared__ double sN[RP * NSMAX * kRmChunk];
  __shared__ int32_t sMask[kRmChunk], sList[kRmChunk];
  __shared__ int32_t scnt[RP * 3];
  __shared__ int32_t s_nl;
  sexp[threadIdx.x] = kExp2TableDev[8 * threadIdx.x];   // kBlock == 256
  const int32_t o0 = blockIdx.y * RP;
  const int32_t np = n_orb - o0 < RP ? n_orb - o0 : RP;
  const int64_t w = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool live = w < n_wav;
  const double lam = wav[live ? w : n_wav - 1];
  const double out = fout_w[live ? w : n_wav - 1];
  // chord counts per phase (stats), by the first workgroup of each phase group
  if (blockIdx.x == 0 && counts) {
    if (threadIdx.x < RP * 3) scnt[threadIdx.x] = 0;
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
  RmStar st{sx, sF, sc, sdir, sexp, 0.0, 0.0, 0, 0};
  if constexpr (!FT) st = rm_stage<UNISTAR>(star, slices, sx, sF, sc, sdir, sexp);
  const int64_t wr = live ? w : n_wav - 1;   // (the table column this lane reads)
  // sigma_s at each of this thread's phases (shift_o * lambda, as getLOSopticalDepth_Batch)
  double sg[RP][NSMAX];
#pragma unroll
  for (int p = 0; p < RP; ++p)
#pragma unroll
    for (int s = 0; s < NSMAX; ++s)
      sg[p][s] = (p < np && s < na) ? sigma_of(tabs[s].shift[o0 + p] * lam, tabs[s]) : 0.0;
  double fstar_uni = 0.0;
  if constexpr (UNISTAR && !FT) fstar_uni = sigma_of(lam / cshift[0], star);
  double loss[RP];
#pragma unroll
  for (int p = 0; p < RP; ++p) loss[p] = 0.0;
  for (int32_t c0 = 0; c0 < n_pr; c0 += kRmChunk) {
    const int nch = n_pr - c0 < kRmChunk ? n_pr - c0 : kRmChunk;
    __syncthreads();
    if (threadIdx.x < kRmChunk) {
      // wave 0: the chunk's masks (active bits 0-7, blocked bits 8-15) and the list of chords with any bit, in
      // chord order (ballot + popcount prefix)
      const int i = threadIdx.x;
      int32_t am = 0, bm = 0;
      if (i < nch) {
        for (int p = 0; p < np; ++p) {
          const int32_t f = flags[(int64_t)(o0 + p) * n_pr + c0 + i];
          am |= (f == 0) << p;
          bm |= (f == 2) << p;
        }
      }
      const int32_t mk = am | (bm << 8);
      sMask[i] = mk;
      const unsigned long long bal = __ballot(mk != 0);
      if (mk != 0) sList[__popcll(bal & ((1ull << i) - 1ull))] = i;
      if (i == 0) s_nl = __popcll(bal);
      if (i < nch) {
        sRho[i] = crho[c0 + i];
        sClv[i] = cclv[c0 + i];
        sSh[i] = cshift[c0 + i];
      }
    }
    for (int i = threadIdx.x; i < na * np * nch; i += kBlock) {
      const int sp = i / nch, c = i - sp * nch;     // sp = s * np + p
      const int s = sp / np, p = sp - s * np;
      sN[(p * NSMAX + s) * kRmChunk + c] = ncol[((int64_t)s * n_orb + o0 + p) * n_pr + c0 + c];
    }
    __syncthreads();
    const int32_t nl = s_nl;
    for (int cg = 0; cg < nl; cg += kRmGroup) {
      double sh[kRmGroup], fsg[kRmGroup];
      int cl[kRmGroup];
#pragma unroll
      for (int u = 0; u < kRmGroup; ++u) {
        cl[u] = sList[cg + u < nl ? cg + u : nl - 1];
        sh[u] = sSh[cl[u]];
      }
      if constexpr (FT) {
#pragma unroll
        for (int u = 0; u < kRmGroup; ++u) fsg[u] = ftab[(int64_t)(c0 + cl[u]) * n_wav + wr];
      } else {
        rm_fstar<UNISTAR>(fsg, lam, sh, st, star, fstar_uni);
      }
#pragma unroll
      for (int u = 0; u < kRmGroup; ++u) {
        if (cg + u >= nl) break;
        const int c = cl[u];
        const double Fc = FT ? fsg[u] : sRho[c] * (fsg[u] * sClv[c]);
        const int32_t mk = __builtin_amdgcn_readfirstlane(sMask[c]);
#pragma unroll
        for (int p = 0; p < RP; ++p) {
          if (p >= np) break;
          if ((mk >> p) & 1) {
            double tau = 0.0;
#pragma unroll
            for (int s = 0; s < NSMAX; ++s)
              if (s < na) tau += sN[(p * NSMAX + s) * kRmChunk + c] * sg[p][s];
            // loss += F (1 - e^-tau)
            loss[p] += Fc;
            if (OCML || !(tau < 700.0 && tau > -700.0)) loss[p] -= Fc * exp(-tau);
            else loss[p] = acc_exp256(loss[p], -Fc, tau * kM256Ln2, sexp);
          } else if ((mk >> (p + 8)) & 1) {
            loss[p] += Fc;                             // blocked at this phase
          }
        }
      }
    }
  }
  if (live) {
#pragma unroll
    for (int p = 0; p < RP; ++p)
      if (p < np) R[(int64_t)(o0 + p) * n_wav + w] = (out - loss[p]) / out;
  }
}

void launch_rm_fout(hipStream_t s, TransitDev& tr) {
  const unsigned nb = (unsigned)((tr.n_wav + kBlock - 1) / kBlock);
  tr.rm_fout.ensure(sizeof(double) * tr.n_wav);
  // the per-chord flux table F(c, w) (a function of the chord grid, the star and the wavelengths only, like Fout):
  // runs then read each listed chord's row instead of looking the stellar spectrum up again (C2 rotating star:
  // 3.7 GB).  PROM_RM_FTAB_MB caps it (default 24,576; 0: off); it also stays within a quarter of the free memory
  const double bytes = 8.0 * (double)tr.n_pr * (double)tr.n_wav;
  static const double cap_mb = [] { const char* e = std::getenv("PROM_RM_FTAB_MB"); return e ? std::atof(e) : 24576.0; }();
  size_t free_b = 0, total_b = 0;
  PROM_HIP(hipMemGetInfo(&free_b, &total_b));
  tr.rm_ftab_ok = !tr.star_uniform && bytes <= cap_mb * 1048576.0 &&
                  bytes + (double)tr.rm_ftab.cap <= 0.25 * ((double)free_b + (double)tr.rm_ftab.cap);
  if (tr.rm_ftab_ok) tr.rm_ftab.ensure((size_t)bytes);
  double* ftab = tr.rm_ftab_ok ? tr.rm_ftab.as<double>() : nullptr;
#define PROM_RMF(UV)                                                                                       \
  hipLaunchKernelGGL((k_rm_fout<UV>), dim3(nb), dim3(kBlock), 0, s, tr.star_tab, tr.rm_slices.as<int32_t>(),  \
                     tr.wav.as<double>(), tr.n_wav, tr.crho.as<double>(), tr.cclv.as<double>(),                  \
                     tr.cshift.as<double>(), tr.n_pr, tr.rm_fout.as<double>(), ftab)
  if (tr.star_uniform) PROM_RMF(true);
  else PROM_RMF(false);
#undef PROM_RMF
  PROM_HIP(hipGetLastError());
}

void launch_tau_rm(hipStream_t s, TransitDev& tr, RunSlot& rs, int32_t na, hipEvent_t* ev) {
    const SigTabDev star = tr.star_tab;
    // phases per workgroup: 2.  Fewer phases hold fewer sigma values and losses in registers (8 phases: 143 VGPRs, 3
    // waves per SIMD; 2: 4+) and list fewer chords per group (the chords blocked or active at one of its phases),
    // at the price of reading a chord once per group it is listed in.  C2 rotating star (tools/rm_bench.py,
    // profiles/r05m_C2_rotating_star.txt): with the flux table 1.71 / 1.22 / 0.74 / 0.81 ms at 8 / 4 / 2 / 1
    // phases; with on-the-fly lookups 2.45 / 2.11 / 1.67 ms at 8 / 4 / 2.  PROM_RM_P (profiling): 1, 2, 4 or 8
    static const int rp_env = [] { const char* e = std::getenv("PROM_RM_P"); return e ? std::atoi(e) : 0; }();
    const int RPv = rp_env == 1 || rp_env == 2 || rp_env == 4 || rp_env == 8 ? rp_env : 2;
    const dim3 g((unsigned)((tr.n_wav + kBlock - 1) / kBlock), (unsigned)((tr.n_orb + RPv - 1) / RPv));
#define PROM_RM(NSV, OC)                                                                                \
  do {                                                                                                  \
    if (tr.star_uniform) { PROM_RM2(NSV, OC, true, false); }                                            \
    else if (tr.rm_ftab_ok) { PROM_RM2(NSV, OC, false, true); }                                         \
    else { PROM_RM2(NSV, OC, false, false); }                                                           \
  } while (0)
#define PROM_RM2(NSV, OC, UV, FTV)                                                                      \
  do {                                                                                                  \
    if (RPv == 1) PROM_RM3(NSV, OC, UV, FTV, 1);                                                        \
    else if (RPv == 2) PROM_RM3(NSV, OC, UV, FTV, 2);                                                   \
    else if (RPv == 4) PROM_RM3(NSV, OC, UV, FTV, 4);                                                   \
    else PROM_RM3(NSV, OC, UV, FTV, 8);                                                                 \
  } while (0)
#define PROM_RM3(NSV, OC, UV, FTV, RPV)                                                                 \
  hipExtLaunchKernelGGL((k_tau_rm<NSV, OC, UV, FTV, RPV>), g, dim3(kBlock), 0, s, ev ? ev[2] : nullptr, ev ? ev[3] : nullptr, 0, \
                        tr.sigtab.as<SigTabDev>(), na, star, tr.rm_slices.as<int32_t>(), tr.wav.as<double>(), \
                        tr.n_wav, tr.crho.as<double>(), tr.cclv.as<double>(), tr.cshift.as<double>(),     \
                        tr.rm_fout.as<double>(), rs.flags.as<int32_t>(), rs.ncol.as<double>(), tr.n_pr, tr.n_orb,                  \
                        tr.count_evals ? rs.counts.as<int32_t>() : nullptr, tr.rm_ftab.as<double>(), rs.R.as<double>())
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
#undef PROM_RM3
}

}  // namespace prom
