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
//     k_columns8  blocking masks, densities evaluated on the fly, column densities
//                 N = sum_x(n chi) dx (numpy pairwise order), tau upper bound -> active /
//                 transparent / blocked  (k_ntot + k_columns when densities must be stored)
//     k_chords    per phase: F_out and transparent sums, compaction of the active chords in chord
//                 order, merging of chords with equal (2^-40) column densities
//     k_tau<NS>   per (phase, wavelength): sigma_s = 10^interp(shift_o * lambda_w) - offset for each
//                 species, then tau over the active chords, exp(-tau), disk sum, ratio
#include "prom_device.h"

namespace prom {

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
    else if (m.kind == PROM_DENSITY_GRIDDED)
      v = grid_density(m, tab, x[ix], cy[ip], cz[ip], bx[sc * n_orb + o], by[sc * n_orb + o]);
    else
      v = density_at(m, x[ix], cy[ip], cz[ip], bx[sc * n_orb + o], by[sc * n_orb + o]);
    ntot[(int64_t)sc * per + i] = v;
  }
}

// Molecular per-sample data (gasProperties.py:925-936): for every molecular slot m and sample
// (o, ip, x): P = (n_tot * k_B) * T clipped below at 1e-4, its bracket on the table's P axis (-1 when
// outside: RegularGridInterpolator's fill, 10^fill - offset = 0), the P weight, and n_abs = n_tot chi.
// molcol[m][o][ip] = sum_x n_abs dx over in-table samples (the chord's bound / sigma_max).
__global__ void k_mol_prep(const MolSlotDev* __restrict__ ms, int32_t n_mol, const double* __restrict__ ntot,
                           int32_t n_x, int32_t n_pr, int32_t n_orb, double delta_x, double4* __restrict__ msmp,
                           int32_t* __restrict__ mnin, double* __restrict__ molcol) {
  const int64_t nc = (int64_t)n_orb * n_pr;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < nc * n_mol;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int32_t m = (int32_t)(c / nc);
    const int64_t cc = c - (int64_t)m * nc;
    const MolSlotDev d = ms[m];
    const double* row = ntot + ((int64_t)d.scenario * nc + cc) * n_x;
    // in-table samples are compacted to the front of the chord's row in sample order as {P weight, n_abs,
    // P bracket, 0}, their count in mnin (out-of-table samples contribute nothing, so the sum over the kept
    // ones is unchanged)
    double col = 0.0;
    const int64_t k0 = ((int64_t)m * nc + cc) * n_x;
    int32_t nin = 0;
    for (int32_t ix = 0; ix < n_x; ++ix) {
      const double n = row[ix];
      double P = n * d.k_B * d.temp;
      P = P < 1e-4 ? 1e-4 : P;
      int64_t i;
      double t;
      const bool in = rgi_bracket(d.P, d.n_p, P, &i, &t);
      if (!in) continue;
      const double na = n * d.chi;
      msmp[k0 + nin] = make_double4(t, na, (double)i, 0.0);
      ++nin;
      col += na * delta_x;
    }
    mnin[(int64_t)m * nc + cc] = nin;
    molcol[(int64_t)m * nc + cc] = col;
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
        bound += molcol[((int64_t)td.slot * n_orb + o) * n_pr + ip] * mol_max_any;
      }
    }
    flags[c] = (bound <= cull) ? 1 : 0;  // NaN bound stays active, like the reference
  }
}

// Per-scenario device view for the streaming column kernel (tab: TABULATED n[(ip*n_orb+o)*n_x+ix], or
// GRIDDED's packed grid).
using ScDev = ScDevHost;

// Blocking masks + column densities + transparency culling in one pass for atomic-only problems with
// n_x <= 64: a group of L = pow2 >= n_x lanes owns one chord, lane i evaluates n(x_i) * chi into LDS,
// lanes 0..7 form numpy's eight pairwise partial sums, lane 0 combines them (loops_utils.h.src order)
// -> N = (0.0 + pairwise_x(n chi)) * delta_x exactly as gasProperties.py:940.  The k_ntot + k_columns
// pair handles molecular terms and n_x > 64.
template <int SPL, int NSIG>
__global__ void __launch_bounds__(kBlock) k_columns8(const ColArgs ca, int32_t n_terms,
                                 const double* __restrict__ x, int32_t n_x,
                                 int32_t n_pr, int32_t n_orb, double delta_x, const double* __restrict__ cy,
                                 const double* __restrict__ cz, const double* __restrict__ bx,
                                 const double* __restrict__ by, const double* __restrict__ planet_y,
                                 double planet_R, int32_t n_moons, const double* __restrict__ moon_y,
                                 const double* __restrict__ moon_R, const double* __restrict__ sig_max,
                                 double cull, double* __restrict__ ncol, int32_t* __restrict__ flags,
                                 const SigTabs4 tabv, const double* __restrict__ wav, int64_t n_wav,
                                 double* __restrict__ sig, float4* __restrict__ tq, int32_t merge_sp,
                                 double nscale_m, int32_t* __restrict__ hcnt, uint8_t* __restrict__ zfl,
                                 int32_t sig_rows, TcPart* __restrict__ tcp) {
  if (hcnt && blockIdx.x == 0 && threadIdx.x < 2) hcnt[threadIdx.x] = 0;   // k_order's heavy-entry counters
  // Eight lanes per chord; lane j holds samples j, j + 8, ..., j + 8 (SPL - 1).  That is numpy's
  // pairwise_sum layout (loops_utils.h.src) for 8 <= n_x < 128: lane j accumulates r[j] = a[j] +
  // a[j+8] + ... sequentially, the eight partial sums combine as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7))
  // through DPP quad permutes and a row shift, and lane 0 adds the n_x % 8 remainder in order.
  PROM_CLK(tk0);
  constexpr int G = kBlock / 8;         // chords per workgroup
  if constexpr (NSIG > 0) {
    // trailing workgroups: sigma_s(shift_{s,o} lambda_w), once per wavelength (sig_rows == 1: no orbital
    // Doppler shift) or once per (phase, wavelength) (sig_rows == n_orb): row r of sig is phase r's
    // chord workgroups [0, cb), padding to cb8 (a multiple of 8), then the sigma workgroups
    const unsigned cb = (unsigned)(((int64_t)n_orb * n_pr + G - 1) / G);
    const unsigned cb8 = (cb + 7u) & ~7u;
    if (blockIdx.x >= cb && blockIdx.x < cb8) return;
    if (blockIdx.x >= cb8) {
      // ... and each 64-wavelength half tile's range of Q = sum_s max(sigma_s / c_s, 0) (float, widened by
      // 2^-20; {-1, 0} when Q is not finite), from which k_order picks the tau windows.  Lanes past
      // n_wav take the last wavelength, as the tau kernels' do.
      // One thread per (row, wavelength): sigma_multi issues the directory loads of all species together,
      // then their node windows.  XCD-aware order: workgroups are dealt to the 8 XCDs round robin, so
      // workgroup b takes item (b % 8) * per + b / 8 of the (wavelength block, row) items, rows fastest:
      // each XCD walks one contiguous wavelength range for all phases and its L2 keeps that range of the
      // tables.
      const int lane = threadIdx.x & 63;
      const int64_t nwb = (n_wav + kBlock - 1) / kBlock;   // sigma workgroups per row
      const int64_t nb = nwb * sig_rows;
      const int64_t per = (nb + 7) / 8;
      const int64_t bp = (int64_t)(blockIdx.x - cb8);
      const int64_t item = (bp & 7) * per + (bp >> 3);
      if (item >= nb) return;
      const int64_t wb = item / sig_rows;
      const int32_t orow = (int32_t)(item - wb * sig_rows);
      const int64_t w = wb * kBlock + threadIdx.x;
      const bool live = w < n_wav;
      const double lam = wav[live ? w : n_wav - 1];
      const int32_t nse = merge_sp ? 1 : NSIG;           // sigma arrays per row
      double tg[NSIG], sv[NSIG];
#pragma unroll
      for (int s = 0; s < NSIG; ++s) tg[s] = tabv.t[s].shift[orow] * lam;
      sigma_multi<NSIG>(tabv, tg, sv);
      double* srow = sig + (int64_t)orow * nse * n_wav;
      double Q = 0.0;
      if (merge_sp) {
        // species merging: the effective absorber's cross-section Y = sum_s chi_s sigma_s
        double Y = 0.0;
        bool z = false;   // some chi_s sigma_s not > 0: an infinite column gives NaN there (inf * 0)
#pragma unroll
        for (int s = 0; s < NSIG; ++s) {
          const double v = tabv.t[s].chi * sv[s];
          z = z || !(v > 0.0);
          Y += v;
        }
        if (live) {
          srow[w] = Y;
          zfl[(int64_t)orow * n_wav + w] = z ? 1 : 0;
        }
        const double qs = Y * nscale_m;
        Q = qs > 0.0 ? qs : 0.0;
      } else {
#pragma unroll
        for (int s = 0; s < NSIG; ++s) {
          if (live) srow[(int64_t)s * n_wav + w] = sv[s];
          const double qs = sv[s] * tabv.t[s].nscale;
          Q += qs > 0.0 ? qs : 0.0;
        }
      }
      const float qf = (float)Q;
      float qh = qf * (1.0f + 0x1p-20f), ql = qf * (1.0f - 0x1p-20f);
      for (int off = 32; off > 0; off >>= 1) {
        qh = fmaxf(qh, __shfl_xor(qh, off, 64));
        ql = fminf(ql, __shfl_xor(ql, off, 64));
      }
      const bool bad = __ballot(!(Q <= 1.0e100)) != 0ull;
      const int64_t n_halves = 2 * ((n_wav + kTW - 1) / kTW);
      const int64_t hw = wb * (kBlock / 64) + (threadIdx.x >> 6);
      if (lane == 0 && hw < n_halves)
        reinterpret_cast<float2*>(tq)[(int64_t)orow * n_halves + hw] =
            bad ? make_float2(-1.0f, 0.0f) : make_float2(ql, qh);
      return;
    }
  }
  const int lane = threadIdx.x & 63;
  const int gl = lane & 7;              // lane within the chord's group
  const int gbase = lane & ~7;
  const int32_t nc = n_orb * n_pr;
  const int32_t c = (int32_t)blockIdx.x * G + (int32_t)threadIdx.x / 8;
  const bool valid = c < nc;
  const int32_t o = valid ? c / n_pr : 0;
  const int32_t ip = valid ? c - o * n_pr : 0;
  const double y = cy[ip], z = cz[ip];
  const double dyp = y - planet_y[o];
  bool blocked = sqrt(dyp * dyp + z * z) < planet_R;
  for (int32_t m = 0; m < n_moons; ++m) {
    const double dym = y - moon_y[m * n_orb + o];
    blocked = blocked || ((dym * dym + z * z) < moon_R[m] * moon_R[m]);
  }
  const int32_t lim = n_x - (n_x % 8);
  const int32_t krem = lim >> 3;        // slot of the remainder samples (lanes 0 .. n_x % 8 - 1)
  double xs[SPL];
#pragma unroll
  for (int k = 0; k < SPL; ++k) {
    const int32_t i = gl + 8 * k;
    xs[k] = i < n_x ? x[i] : 0.0;
  }
  double bound = 0.0;
  double n_last = 0.0;   // (the last term's column: the transmission-curve path has one term)
  double nv[SPL];
  int32_t cur_sc = -1;
#pragma unroll
  for (int32_t t = 0; t < 8; ++t) {
    if (t >= n_terms) break;
    const TermDev td = ca.t[t];
    if (td.scenario != cur_sc) {   // one density evaluation per scenario, shared by its constituents
      cur_sc = td.scenario;
      const ScDev sc = ca.sc[cur_sc & 3];
      const double bxo = bx[cur_sc * n_orb + o], byo = by[cur_sc * n_orb + o];
#pragma unroll
      for (int k = 0; k < SPL; ++k) {
        const int32_t i = gl + 8 * k;
        nv[k] = 0.0;
        if (valid && !blocked && i < n_x)
          nv[k] = sc.m.kind == PROM_DENSITY_GRIDDED ? grid_density(sc.m, sc.tab, xs[k], y, z, bxo, byo)
                  : sc.tab ? sc.tab[((int64_t)ip * n_orb + o) * n_x + i] : density_at(sc.m, xs[k], y, z, bxo, byo);
      }
    }
    double av[SPL];
#pragma unroll
    for (int k = 0; k < SPL; ++k) av[k] = (gl + 8 * k < n_x) ? nv[k] * td.chi : 0.0;
    double res;
    if (n_x < 8) {
      res = 0.0;
      for (int32_t i = 0; i < n_x; ++i) res += __shfl(av[0], gbase + i, 64);
    } else {
      double r = av[0];
#pragma unroll
      for (int k = 1; k < SPL; ++k)
        if (8 * k < lim) r += av[k];
      double t1 = dpp_mov<0xB1>(r);        // quad_perm [1,0,3,2]: partner lane ^ 1
      r = r + t1;
      t1 = dpp_mov<0x4E>(r);               // quad_perm [2,3,0,1]: partner lane ^ 2
      r = r + t1;
      t1 = dpp_mov<0x104>(r);              // row_shl:4: lanes 0-3 (8-11) read 4-7 (12-15)
      res = r + t1;
      double rem = 0.0;
#pragma unroll
      for (int k = 0; k < SPL; ++k)
        if (k == krem) rem = av[k];
      // lane 0 of the group adds the remainder samples lim .. n_x-1 (lanes 0 .. n_x-lim-1) in order
      const int32_t nrem = n_x - lim;
      if (nrem > 0) res += rem;
      if (nrem > 1) res += dpp_mov<0x101>(rem);
      if (nrem > 2) res += dpp_mov<0x102>(rem);
      if (nrem > 3) res += dpp_mov<0x103>(rem);
      if (nrem > 4) res += dpp_mov<0x104>(rem);
      if (nrem > 5) res += dpp_mov<0x105>(rem);
      if (nrem > 6) res += dpp_mov<0x106>(rem);
    }
    const double N = blocked ? 0.0 : (0.0 + res) * delta_x;
    if (gl == 0 && valid) ncol[((int64_t)td.slot * n_orb + o) * n_pr + ip] = N;
    bound += N * sig_max[td.slot];
    n_last = N;
  }
  const int32_t fcls = blocked ? 2 : ((bound <= cull) ? 1 : 0);
  if (gl == 0 && valid) flags[c] = fcls;
  if (tcp) {
    // transmission curves (one term, n_pr % 32 == 0: the workgroup's 32 chords belong to one phase): the group's
    // max / min over its active finite columns and counts, folded by wave 0 (order-independent)
    __shared__ double s_n[G];
    __shared__ int32_t s_f[G];
    if (gl == 0) {
      s_n[threadIdx.x / 8] = n_last;
      s_f[threadIdx.x / 8] = valid ? fcls : 3;
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      const int li = threadIdx.x & (G - 1);
      const bool own = threadIdx.x < G;
      const int32_t f = own ? s_f[li] : 3;
      const double n = s_n[li];
      const bool act = f == 0, fin = __builtin_isfinite(n);
      double mx = (act && fin) ? n : 0.0;
      double mn = (act && fin && n > 0.0) ? n : __builtin_inf();
      int32_t ca = act ? 1 : 0, ct = f == 1 ? 1 : 0, cb = f == 2 ? 1 : 0, cn = (act && !fin) ? 1 : 0;
      for (int off = 32; off > 0; off >>= 1) {
        mx = fmax(mx, __shfl_xor(mx, off, 64));
        mn = fmin(mn, __shfl_xor(mn, off, 64));
        ca += __shfl_xor(ca, off, 64);
        ct += __shfl_xor(ct, off, 64);
        cb += __shfl_xor(cb, off, 64);
        cn += __shfl_xor(cn, off, 64);
      }
      const int32_t c0 = (int32_t)blockIdx.x * G;
      if (threadIdx.x == 0 && c0 < nc) {
        TcPart pv;
        pv.nmax = mx; pv.nmin = mn; pv.nact = ca; pv.ntr = ct; pv.nbl = cb; pv.nnf = cn;
        tcp[c0 / G] = pv;   // (phase c0 / n_pr, group (c0 % n_pr) / 32: consecutive)
      }
    }
  }
#ifdef PROM_TRACE
  {
    const int64_t wv = 600000 + 2 * ((int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6));
    PROM_ACC(wv + 0, clock64() - tk0);
    PROM_ACC(wv + 1, 1);
  }
#endif
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
__device__ __forceinline__ unsigned long long mkey(double v) {
  return __builtin_bit_cast(unsigned long long, v) >> 12;
}

// ---- per-phase chord bookkeeping: compaction + merging in one workgroup ----------------------------
// Pass 1: F_out sum, transparent sum, counts, non-finite check.  Pass 2: compaction of the active
// chords in chord order into records {F_out / F_out_sum, N_0..N_{S-1}} (recs, act_ip: the exact path
// and the unmerged fast path).  Pass 3 (merging, see k_merge's comment for the bound): LDS bitonic sort
// of (key_0, key_1, position), group heads, one merged record per group (mrecs).
// counts[o * kCnt] = {active, transparent, blocked, nonfinite, records, sorted/merged, windowed, 0}.
constexpr int kChordBlock = 1024;
constexpr int kChordMergeMax = 2048;

// inclusive/exclusive scan of v over the workgroup; returns the exclusive prefix, *total = sum
__device__ __forceinline__ int32_t block_excl_scan(int32_t v, int32_t* wsum, int32_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int32_t inc = v;
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t u = __shfl_up(inc, off, 64);
    if (lane >= off) inc += u;
  }
  __syncthreads();
  if (lane == 63) wsum[wid] = inc;
  __syncthreads();
  int32_t wb = 0, tot = 0;
  for (int w = 0; w < kChordBlock / 64; ++w) {
    if (w < wid) wb += wsum[w];
    tot += wsum[w];
  }
  *total = tot;
  return wb + inc - v;
}

constexpr int kChordPer = 4;   // chords per thread held in registers (n_pr <= 4096 in one sweep)

__global__ void __launch_bounds__(kChordBlock) k_chords(const int32_t* __restrict__ flags,
                                                        const double* __restrict__ fout,
                                                        const double* __restrict__ ncol, int32_t n_atoms,
                                                        int32_t n_pr, int32_t n_orb, int32_t merge,
                                                        double* __restrict__ recs,
                                                        int32_t* __restrict__ act_ip,
                                                        double* __restrict__ mrecs,
                                                        int32_t* __restrict__ counts,
                                                        double* __restrict__ tfrac,
                                                        double* __restrict__ fsum) {
  __shared__ double redd[2][kChordBlock / 64];
  __shared__ int32_t redi[kChordBlock / 64];
  __shared__ int32_t redc[3][kChordBlock / 64];
  __shared__ double Fl[kChordMergeMax];
  __shared__ unsigned long long k0[kChordMergeMax];
  __shared__ unsigned long long k1[kChordMergeMax];
  __shared__ int32_t idx[kChordMergeMax];
  __shared__ int32_t gid[kChordMergeMax];
  const int32_t o = blockIdx.x;
  const int32_t stride = 1 + n_atoms;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // this thread's contiguous chords: [c_lo, c_hi); sweeps of kChordBlock*kChordPer chords
  const int32_t per_sweep = kChordBlock * kChordPer;
  double fpart = 0.0, tpart = 0.0;
  int32_t ntr = 0, nbl = 0, nnf = 0;
  for (int32_t sw = 0; sw < n_pr; sw += per_sweep) {
    const int32_t lo = sw + threadIdx.x * kChordPer;
#pragma unroll
    for (int k = 0; k < kChordPer; ++k) {
      const int32_t ip = lo + k;
      if (ip >= n_pr || ip >= sw + per_sweep) break;
      const int32_t f = flags[(int64_t)o * n_pr + ip];
      const double fo = fout[ip];
      fpart += fo;
      if (f == 1) { tpart += fo; ++ntr; }
      if (f == 2) ++nbl;
      if (f == 0)
        for (int32_t s = 0; s < n_atoms; ++s)
          if (!__builtin_isfinite(ncol[((int64_t)s * n_orb + o) * n_pr + ip])) { ++nnf; break; }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    fpart += __shfl_down(fpart, off, 64);
    tpart += __shfl_down(tpart, off, 64);
    ntr += __shfl_down(ntr, off, 64);
    nbl += __shfl_down(nbl, off, 64);
    nnf += __shfl_down(nnf, off, 64);
  }
  if (lane == 0) {
    redd[0][wid] = fpart; redd[1][wid] = tpart;
    redc[0][wid] = ntr; redc[1][wid] = nbl; redc[2][wid] = nnf;
  }
  __syncthreads();
  double fs = 0.0, ts = 0.0;
  ntr = nbl = nnf = 0;
  for (int w = 0; w < kChordBlock / 64; ++w) {
    fs += redd[0][w]; ts += redd[1][w];
    ntr += redc[0][w]; nbl += redc[1][w]; nnf += redc[2][w];
  }
  // compaction in chord order
  int32_t base = 0;
  for (int32_t sw = 0; sw < n_pr; sw += per_sweep) {
    const int32_t lo = sw + threadIdx.x * kChordPer;
    int32_t mine = 0;
#pragma unroll
    for (int k = 0; k < kChordPer; ++k) {
      const int32_t ip = lo + k;
      if (ip < n_pr && flags[(int64_t)o * n_pr + ip] == 0) ++mine;
    }
    int32_t tot;
    int32_t pos = base + block_excl_scan(mine, redi, &tot);
#pragma unroll
    for (int k = 0; k < kChordPer; ++k) {
      const int32_t ip = lo + k;
      if (ip >= n_pr || flags[(int64_t)o * n_pr + ip] != 0) continue;
      act_ip[(int64_t)o * n_pr + pos] = ip;
      double* r = recs + ((int64_t)o * n_pr + pos) * stride;
      const double F = fout[ip] / fs;
      r[0] = F;
      double n0 = 0.0, n1 = 0.0;
      for (int32_t s = 0; s < n_atoms; ++s) {
        const double v = ncol[((int64_t)s * n_orb + o) * n_pr + ip];
        r[1 + s] = v;
        if (s == 0) n0 = v;
        if (s == 1) n1 = v;
      }
      if (pos < kChordMergeMax) {
        Fl[pos] = F;
        k0[pos] = mkey(n0);
        k1[pos] = n_atoms > 1 ? mkey(n1) : 0ull;
        idx[pos] = pos;
      }
      ++pos;
    }
    base += tot;
  }
  const int32_t n = base;
  const bool do_merge = merge && n >= 2 && n <= kChordMergeMax && nnf == 0;
  int32_t G = n;
  if (do_merge) {
    int32_t P = 1;
    while (P < n) P <<= 1;
    for (int32_t i = n + threadIdx.x; i < P; i += kChordBlock) { k0[i] = ~0ull; k1[i] = ~0ull; idx[i] = 0x7fffffff; }
    __syncthreads();
    for (int32_t size = 2; size <= P; size <<= 1) {
      for (int32_t st = size >> 1; st > 0; st >>= 1) {
        for (int32_t t = threadIdx.x; t < P / 2; t += kChordBlock) {
          const int32_t i = 2 * t - (t & (st - 1));
          const int32_t j = i + st;
          const bool up = (i & size) == 0;
          const unsigned long long a0 = k0[i], b0 = k0[j], a1 = k1[i], b1 = k1[j];
          const int32_t ai = idx[i], bi = idx[j];
          const bool gt = (a0 > b0) || (a0 == b0 && (a1 > b1 || (a1 == b1 && ai > bi)));
          if (gt == up) {
            k0[i] = b0; k0[j] = a0; k1[i] = b1; k1[j] = a1; idx[i] = bi; idx[j] = ai;
          }
        }
        __syncthreads();
      }
    }
    const double* orec = recs + (int64_t)o * n_pr * stride;
    int32_t gbase = 0;
    for (int32_t c0 = 0; c0 < n; c0 += kChordBlock) {
      const int32_t i = c0 + threadIdx.x;
      bool head = false;
      if (i < n) {
        head = (i == 0) || k0[i] != k0[i - 1] || k1[i] != k1[i - 1];
        if (!head && n_atoms > 2) {
          const double* a = orec + (int64_t)idx[i] * stride;
          const double* b = orec + (int64_t)idx[i - 1] * stride;
          for (int32_t s = 2; s < n_atoms && !head; ++s) head = mkey(a[1 + s]) != mkey(b[1 + s]);
        }
      }
      int32_t tot;
      const int32_t rank = block_excl_scan(head ? 1 : 0, redi, &tot);
      if (i < n) gid[i] = gbase + rank + (head ? 0 : -1);
      gbase += tot;
    }
    __syncthreads();
    G = gbase;
    double* mo = mrecs + (int64_t)o * n_pr * stride;
    for (int32_t i = threadIdx.x; i < n; i += kChordBlock) {
      if (i > 0 && gid[i] == gid[i - 1]) continue;
      double F = Fl[idx[i]];
      for (int32_t j = i + 1; j < n && gid[j] == gid[i]; ++j) F += Fl[idx[j]];
      const double* a = orec + (int64_t)idx[i] * stride;
      double* r = mo + (int64_t)gid[i] * stride;
      r[0] = F;
      for (int32_t s = 0; s < n_atoms; ++s) r[1 + s] = a[1 + s];
    }
  }
  if (threadIdx.x == 0) {
    tfrac[o] = ts / fs;
    fsum[o] = fs;
    counts[o * kCnt + 0] = n;
    counts[o * kCnt + 1] = ntr;
    counts[o * kCnt + 2] = nbl;
    counts[o * kCnt + 3] = nnf;
    counts[o * kCnt + 4] = G;
    counts[o * kCnt + 5] = do_merge ? 1 : 0;
    counts[o * kCnt + 6] = 0;
    counts[o * kCnt + 7] = 0;
  }
}


// One workgroup per phase, few dependent steps (2 global round trips, ~8 workgroup barriers for
// phases with <= 1024 active chords):
//  1. every thread loads its strided chords (flags, F_out, N_s) -- one round trip per 4096 chords --
//     classifies them, writes the sort key (b descending, chord index) of each active chord at its
//     thread-major compaction position; one combined workgroup scan/reduction gives positions,
//     counts, the F_out sum and the transparent sum;
//  2. phases with non-finite columns (exact path) or more than kWinMax active chords, or with neither
//     merging nor windows requested: chord-order-free compaction into recs/act_ip instead;
//  3. keys sorted in LDS: rank sort (<= 1024 keys: each key's rank = number of smaller keys, counted
//     against LDS broadcasts) or bitonic;
//  4. each thread fetches the columns of its ceil(n / kWBlock) consecutive sorted positions (one trip),
//     forms b, a, F and group heads (equal 2^-40 keys of every species when merge != 0);
//  5. one combined workgroup scan: group ids (prefix sum of heads), A (prefix min of a), B (suffix max
//     of b) and the K suffix moments;
//  6. each group head writes its record (summed weight, head's columns), moments and envelopes;
//     threshold tables are searched in LDS.
// counts[o * kCnt] = {active, transparent, blocked, nonfinite, records, sorted, windowed, 0}.
constexpr int kLD = kWinMax / kWBlock;              // strided chords per thread and sweep
constexpr int kRankMax = 2 * kWBlock;               // rank sort up to this many keys
#ifndef PROM_ORD_EXP
#define PROM_ORD_EXP 0   // profiling only: skip parts of k_order's record step (wrong results)
#endif
constexpr int kSlotBin = 128;                       // slot sort when no slot holds more than this many keys
constexpr int kPayMax = 2048;                       // stage columns in LDS up to this many chords

template <int NS>
__global__ void __launch_bounds__(kWBlock) k_order(const int32_t* __restrict__ flags,
                                                   const double* __restrict__ fout,
                                                   const double* __restrict__ ncol, int32_t n_pr,
                                                   int32_t n_orb, int32_t merge, int32_t window,
                                                   const SigTabs4 tabv,
                                                   double* __restrict__ recs,
                                                   int32_t* __restrict__ act_ip,
                                                   double* __restrict__ mrecs,
                                                   int32_t* __restrict__ counts,
                                                   double* __restrict__ tfrac,
                                                   double* __restrict__ fsum,
                                                   int32_t* __restrict__ wenv,
                                                   double* __restrict__ wmom,
                                                   double btail) {
  constexpr Monos<NS> M{};
  constexpr int K = Monos<NS>::K;
  constexpr int NW = kWBlock / 64;
  constexpr int ST = 1 + NS;
  __shared__ unsigned long long skey[kWinMax];   // sort keys: 2^-30 buckets of b, compaction position
  __shared__ double sF[kWinMax];                 // F_out: by compaction position (payload in LDS) or by
                                                 // sorted position (columns fetched from HBM)
  constexpr int PAY = NS == 1 ? kWinMax : (NS >= 4 ? kPayMax / 2 : kPayMax);   // LDS budget (160 KiB)
  __shared__ double sN[NS][PAY];                 // columns by compaction position (n <= PAY)
  __shared__ int32_t sIp[kWinMax];               // chord index by compaction position
  __shared__ unsigned char sHead[kWinMax];
  __shared__ int32_t hB[kEnvN + 2], hA[kEnvN + 2];   // envelope histograms (threshold tables)
  __shared__ int32_t pi_[NW][5];
  __shared__ double pd_[NW][2];
  __shared__ double pm_[NW][K + 2];
  __shared__ int32_t pg_[NW];
  const int32_t o = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int32_t* fl = flags + (int64_t)o * n_pr;
  const int64_t nstride = (int64_t)n_orb * n_pr;
  const double* nc0 = ncol + (int64_t)o * n_pr;
  double cs[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) cs[s] = tabv.t[s].ncoef;

  PROM_TS(o * 16 + 0);
  for (int32_t i = tid; i < kEnvN + 2; i += kWBlock) { hB[i] = 0; hA[i] = 0; }
  // ---- 1. load, classify, keys, combined scan/reduction.  Active chords whose bound b is below btail
  //         (b Q < the tail epsilon at every wavelength of the problem) are tail records everywhere: they
  //         are compacted behind the others, unsorted (single sweep only)
  const bool part = n_pr <= kWinMax && btail > 0.0;
  double fs = 0.0, ts = 0.0;
  int32_t nact = 0, ntr = 0, nbl = 0, nnf = 0, ncand = 0;
  for (int32_t sw = 0; sw < n_pr; sw += kWinMax) {
    int32_t f[kLD];
    double fo[kLD], nv[kLD][NS], bk[kLD];
#pragma unroll
    for (int k = 0; k < kLD; ++k) {
      const int32_t ip = sw + tid + k * kWBlock;
      const bool in = ip < n_pr;
      f[k] = in ? fl[ip] : 3;
      fo[k] = in ? fout[ip] : 0.0;
#pragma unroll
      for (int s = 0; s < NS; ++s) nv[k][s] = in ? nc0[s * nstride + ip] : 0.0;
    }
    PROM_TS(o * 16 + 7);
    double fp = 0.0, tp = 0.0;
    int32_t c[5] = {0, 0, 0, 0, 0};   // active (not tail), transparent, blocked, nonfinite, tail
    uint32_t tailbits = 0;
#pragma unroll
    for (int k = 0; k < kLD; ++k) {
      bk[k] = 0.0;
      if (f[k] == 3) continue;
      fp += fo[k];
      if (f[k] == 1) { tp += fo[k]; ++c[1]; }
      else if (f[k] == 2) ++c[2];
      else {
        double b = 0.0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          if (!__builtin_isfinite(nv[k][s])) { ++c[3]; break; }
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const double v = nv[k][s] * cs[s];
          b = v > b ? v : b;
        }
        b = b < 1.0 ? b : 1.0;   // NaN -> 1.0 (such phases take the unsorted path anyway)
        bk[k] = b;
        if (part && b < btail) { ++c[4]; tailbits |= 1u << k; }
        else ++c[0];
      }
    }
    // combined: prefixes of the candidate and tail counts, wavefront totals of everything (DPP scans); the
    // five counts (<= kLD per lane, <= 64 kLD = 512 per wavefront) travel as 10-bit fields of two scans
    static_assert(64 * kLD < 1024, "10-bit count fields");
    const int32_t pa = wave_prefix<int32_t>(c[0] | (c[4] << 10) | (c[1] << 20), OpAdd());
    const int32_t pb = lane_read(wave_prefix<int32_t>(c[2] | (c[3] << 10), OpAdd()), 63);
    const int32_t pa63 = lane_read(pa, 63);
    const int32_t inc = pa & 1023, inct = (pa >> 10) & 1023;
    const double fpw = lane_read(wave_prefix<double>(fp, OpAdd()), 63);
    const double tpw = lane_read(wave_prefix<double>(tp, OpAdd()), 63);
    const int32_t c1w = (pa63 >> 20) & 1023, c2w = pb & 1023, c3w = (pb >> 10) & 1023;
    lds_barrier();
    if (lane == 63) { pi_[wid][0] = inc; pi_[wid][4] = inct; }
    if (lane == 0) {
      pi_[wid][1] = c1w; pi_[wid][2] = c2w; pi_[wid][3] = c3w;
      pd_[wid][0] = fpw; pd_[wid][1] = tpw;
    }
    lds_barrier();
    int32_t sc_ = 0;   // candidates of this sweep
    for (int w = 0; w < NW; ++w) sc_ += pi_[w][0];
    int32_t pos = nact + inc - c[0];
    int32_t post = nact + sc_ + inct - c[4];
    for (int w = 0; w < NW; ++w) {
      if (w < wid) { pos += pi_[w][0]; post += pi_[w][4]; }
      nact += pi_[w][0] + pi_[w][4]; ntr += pi_[w][1]; nbl += pi_[w][2]; nnf += pi_[w][3];
      fs += pd_[w][0]; ts += pd_[w][1];
    }
    ncand += sc_;
#pragma unroll
    for (int k = 0; k < kLD; ++k) {
      if (f[k] != 0) continue;
      const bool tl = (tailbits >> k) & 1u;
      const int32_t pk = tl ? post : pos;
      if (pk < kWinMax) {
        const unsigned long long d =
            (__builtin_bit_cast(unsigned long long, 1.0) - __builtin_bit_cast(unsigned long long, bk[k])) >> 22;
        skey[pk] = (d << 24) | (unsigned long long)pk;
        sIp[pk] = sw + tid + k * kWBlock;
        if (pk < PAY) {
          sF[pk] = fo[k];
#pragma unroll
          for (int s = 0; s < NS; ++s) sN[s][pk] = nv[k][s];
        }
      }
      if (tl) ++post; else ++pos;
    }
  }
  lds_barrier();   // keys visible to the sort
  PROM_TS(o * 16 + 1);
  const bool sorted = nnf == 0 && nact <= kWinMax && (merge || window);
  int32_t G = nact;
  int32_t dbg_word = 0;   // counts[7]: candidates | sort path << 13 | largest slot << 16
  if (!sorted) {
    // ---- 2. compaction into recs / act_ip (thread-major order, deterministic)
    int32_t base = 0;
    for (int32_t sw = 0; sw < n_pr; sw += kWinMax) {
      int32_t f[kLD];
      int32_t mine = 0;
#pragma unroll
      for (int k = 0; k < kLD; ++k) {
        const int32_t ip = sw + tid + k * kWBlock;
        f[k] = ip < n_pr ? fl[ip] : 3;
        mine += f[k] == 0 ? 1 : 0;
      }
      int32_t tot;
      int32_t pos = base + wg_excl_prefix<int32_t>(mine, OpAdd(), 0, pg_, &tot);
#pragma unroll
      for (int k = 0; k < kLD; ++k) {
        if (f[k] != 0) continue;
        const int32_t ip = sw + tid + k * kWBlock;
        act_ip[(int64_t)o * n_pr + pos] = ip;
        double* r = recs + ((int64_t)o * n_pr + pos) * ST;
        r[0] = fout[ip] / fs;
#pragma unroll
        for (int s = 0; s < NS; ++s) r[1 + s] = nc0[s * nstride + ip];
        ++pos;
      }
      base += tot;
    }
  } else {
    const int32_t n = nact;
    const int32_t n_all = n;
    // ---- 3. sort the candidates [0, ncand); tail records [ncand, n) keep their compaction order
    {
    const int32_t n = ncand;
    // Slot sort (candidates spread over the 1/8-octave slots of b): the key's slot is d >> 27 =
    // (bits(1.0) - bits(b)) >> 49 with bits(b) >> 22 = d quantised inside one slot (2^22 divides 2^49), so
    // ordering by (slot, key) IS the order of the keys: a counting sort over the slots (LDS histogram and
    // cursors in hB / hA, the keys scattered by slot back into skey from registers), then each key's rank
    // among its slot's keys, the lanes of a wavefront reading the same few slots (broadcasts).  The
    // O(n^2 / threads) rank sort and the merge sort's dependent, bank-conflicted binary searches took
    // 11-18 us of C3's 36 us k_order (~1,500 candidates per phase, profiles/r03*_trace_C3.txt).
    constexpr int SQ = kWinMax / kWBlock;
    bool slot_sorted = false;
    int32_t dbg_path = 0, dbg_cmax = 0;
    bool crowded = false;
    if (n > 64) {
      __shared__ int32_t s_flag;
      if (tid == 0) s_flag = 0;
      lds_barrier();
      unsigned long long kk[SQ];
#pragma unroll
      for (int q = 0; q < SQ; ++q) {
        const int32_t i = tid + q * kWBlock;
        kk[q] = i < n ? skey[i] : 0ull;
        if (i < n) {
          const int64_t sk = (int64_t)(kk[q] >> 51);   // d >> 27 (the key is d << 24 | position)
          if (sk >= kEnvN) s_flag = 1;
          else atomicAdd(&hB[sk], 1);
        }
      }
      lds_barrier();
      if (!s_flag) {
        // exclusive scan of the kEnvN slot counts (kEnvN / kWBlock per thread) -> cursors in hA
        constexpr int PS = kEnvN / kWBlock;
        int32_t c[PS], run = 0, cmax = 0;
#pragma unroll
        for (int k = 0; k < PS; ++k) { c[k] = hB[tid * PS + k]; run += c[k]; cmax = c[k] > cmax ? c[k] : cmax; }
        int32_t tot;
        const int32_t base = wg_excl_prefix<int32_t>(run, OpAdd(), 0, pg_, &tot);
        int32_t acc = base;
#pragma unroll
        for (int k = 0; k < PS; ++k) { hA[tid * PS + k] = acc; hB[tid * PS + k] = acc; acc += c[k]; }
        if (cmax > 0) atomicMax(&hB[kEnvN + 1], cmax);
        lds_barrier();
        dbg_cmax = hB[kEnvN + 1];
        crowded = dbg_cmax > kSlotBin;   // a crowded slot: the rank step would be quadratic in it
      }
      if (!s_flag && !crowded) {
        // scatter by slot (arrival order within a slot), then rank inside the slot by key
#pragma unroll
        for (int q = 0; q < SQ; ++q)
          if (tid + q * kWBlock < n) skey[atomicAdd(&hA[(int32_t)(kk[q] >> 51)], 1)] = kk[q];
        lds_barrier();
        int32_t dst[SQ];
#pragma unroll
        for (int q = 0; q < SQ; ++q) {
          const int32_t i = tid + q * kWBlock;
          dst[q] = -1;
          if (i >= n) continue;
          const unsigned long long k = skey[i];
          const int32_t sk = (int32_t)(k >> 51);
          const int32_t a = hB[sk], b = hA[sk];   // the slot's segment [a, b) (hA: the cursors' end)
          int32_t r = 0, j = a;
          for (; j + 4 <= b; j += 4) {
            const unsigned long long x0 = skey[j], x1 = skey[j + 1], x2 = skey[j + 2], x3 = skey[j + 3];
            r += (x0 < k) + (x1 < k) + (x2 < k) + (x3 < k);
          }
          for (; j < b; ++j) r += skey[j] < k;
          kk[q] = k;
          dst[q] = a + r;
        }
        lds_barrier();   // every rank counted before any key moves
#pragma unroll
        for (int q = 0; q < SQ; ++q)
          if (dst[q] >= 0) skey[dst[q]] = kk[q];
        slot_sorted = true;
      }
      lds_barrier();
      for (int32_t i = tid; i < kEnvN + 2; i += kWBlock) { hB[i] = 0; hA[i] = 0; }   // (the envelope histograms)
      lds_barrier();
    }
    dbg_path = slot_sorted ? 1 : (n <= kRankMax ? 2 : 3);
    dbg_word = n | (dbg_path << 13) | ((dbg_cmax < 2047 ? dbg_cmax : 2047) << 16);
    if (slot_sorted) {
    } else if (n <= kRankMax) {
      // rank = number of smaller keys (keys are unique: they carry the chord index); only the
      // wavefronts holding keys count, against LDS broadcasts
      const int32_t i0 = tid, i1 = tid + kWBlock;
      const bool has0 = i0 < n, has1 = i1 < n;
      const unsigned long long k0 = has0 ? skey[i0] : ~0ull;
      const unsigned long long k1 = has1 ? skey[i1] : ~0ull;
      int32_t r0 = 0, r1 = 0;
      // keys past n read as ~0 (never smaller); 16 broadcast loads in flight per step
      for (int32_t i = n + tid; i < ((n + 15) & ~15); i += kWBlock) skey[i] = ~0ull;
      lds_barrier();
      const int32_t n16 = (n + 15) & ~15;
      if (n > kWBlock) {
        for (int32_t j = 0; j < n16; j += 16) {
          unsigned long long a[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) a[q] = skey[j + q];
#pragma unroll
          for (int q = 0; q < 16; ++q) { r0 += a[q] < k0; r1 += a[q] < k1; }
        }
      } else if (__builtin_amdgcn_readfirstlane(tid) < n) {
        for (int32_t j = 0; j < n16; j += 16) {
          unsigned long long a[16];
#pragma unroll
          for (int q = 0; q < 16; ++q) a[q] = skey[j + q];
#pragma unroll
          for (int q = 0; q < 16; ++q) r0 += a[q] < k0;
        }
      }
      lds_barrier();
      if (has0) skey[r0] = k0;
      if (has1) skey[r1] = k1;
      lds_barrier();
    } else {
      // merge sort in place (keys are unique): thread t owns positions [8t, 8t + 8); its eight keys are
      // sorted in registers, then runs of L = 8, 16, .. P/2 merge pairwise: a key's position in the
      // merged run is its index in its own run plus the number of smaller keys in the partner run (a
      // branchless binary search in LDS, the eight keys interleaved); 9 passes of 2 barriers at P = 4096
      constexpr int KP = kWinMax / kWBlock;
      static_assert(KP == 8, "eight keys per thread");
      int32_t P = 8;
      while (P < n) P <<= 1;
      // padding keys: unique (the merge ranks assume it) and above every real key (<= 0xffc0... | pos)
      for (int32_t i = n + tid; i < P; i += kWBlock) skey[i] = 0xffffffffffff0000ull | (unsigned)i;
      lds_barrier();
      const int32_t p0 = KP * tid;
      const bool own = p0 < P;
      unsigned long long k[KP];
#pragma unroll
      for (int q = 0; q < KP; ++q) k[q] = own ? skey[p0 + q] : ~0ull;
      // Batcher's odd-even merge sort network for 8 keys (19 compare-exchanges)
      auto cx = [&](int a, int b) {
        const unsigned long long x = k[a], y = k[b];
        k[a] = x < y ? x : y;
        k[b] = x < y ? y : x;
      };
      cx(0, 1); cx(2, 3); cx(4, 5); cx(6, 7);
      cx(0, 2); cx(1, 3); cx(4, 6); cx(5, 7);
      cx(1, 2); cx(5, 6);
      cx(0, 4); cx(1, 5); cx(2, 6); cx(3, 7);
      cx(2, 4); cx(3, 5);
      cx(1, 2); cx(3, 4); cx(5, 6);
      lds_barrier();   // every chunk loaded before any sorted chunk is stored
      if (own) {
#pragma unroll
        for (int q = 0; q < KP; ++q) skey[p0 + q] = k[q];
      }
      lds_barrier();
      for (int32_t L = KP; L < P; L <<= 1) {
        const int32_t base = p0 & ~(2 * L - 1);
        const bool left = (p0 & L) == 0;
        const int32_t ps = left ? base + L : base;           // partner run [ps, ps + L)
        const int32_t idx = p0 - (left ? base : base + L);   // index of k[0] in its own run
        int32_t lo[KP];
#pragma unroll
        for (int q = 0; q < KP; ++q) lo[q] = 0;
        if (own) {
          for (int32_t st = L >> 1; st > 0; st >>= 1) {
#pragma unroll
            for (int q = 0; q < KP; ++q)
              if (skey[ps + lo[q] + st - 1] < k[q]) lo[q] += st;
          }
#pragma unroll
          for (int q = 0; q < KP; ++q)
            if (lo[q] == L - 1 && skey[ps + L - 1] < k[q]) lo[q] = L;
        }
        lds_barrier();   // every search done before any key moves
        if (own) {
#pragma unroll
          for (int q = 0; q < KP; ++q) skey[base + idx + q + lo[q]] = k[q];
        }
        lds_barrier();
        if (own) {
#pragma unroll
          for (int q = 0; q < KP; ++q) k[q] = skey[p0 + q];
        }
      }
    }
    }
    // tail keys: only their compaction position (low 24 bits) is read from here on; the sort's padding
    // may have overwritten some, so they are rewritten
    lds_barrier();
    for (int32_t i = ncand + tid; i < n_all; i += kWBlock) skey[i] = (unsigned long long)i;
    lds_barrier();
    PROM_TS(o * 16 + 2);
    // ---- 4. this thread's sorted positions [i0, i0 + cnt)
    const int32_t per = (n + kWBlock - 1) / kWBlock;   // <= kWPer
    const int32_t i0 = min(n, tid * per);
    const int32_t cnt = min(n, i0 + per) - i0;
    double Nv[kWPer][NS], Fv[kWPer], bv[kWPer], av[kWPer];
    double Np[NS];
    const bool lds_pay = n <= PAY;   // columns and F_out staged in LDS at compaction
    {
      const int32_t pp = i0 > 0 ? (int32_t)(skey[i0 - 1] & 0xffffffull) : 0;
      if (lds_pay) {
#pragma unroll
        for (int s = 0; s < NS; ++s) Np[s] = (i0 > 0 && cnt > 0) ? sN[s][pp] : 0.0;
      } else {
        const int32_t ipp = sIp[pp];
#pragma unroll
        for (int s = 0; s < NS; ++s) Np[s] = (i0 > 0 && cnt > 0) ? nc0[s * nstride + ipp] : 0.0;
      }
    }
    if (lds_pay) {
#pragma unroll
      for (int k = 0; k < kWPer; ++k) {
        const int32_t pk = k < cnt ? (int32_t)(skey[i0 + k] & 0xffffffull) : 0;
        Fv[k] = k < cnt ? sF[pk] : 0.0;
#pragma unroll
        for (int s = 0; s < NS; ++s) Nv[k][s] = k < cnt ? sN[s][pk] : 0.0;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kWPer; ++k) {
        const int32_t ip = k < cnt ? sIp[(int32_t)(skey[i0 + k] & 0xffffffull)] : 0;
        Fv[k] = k < cnt ? fout[ip] : 0.0;
#pragma unroll
        for (int s = 0; s < NS; ++s) Nv[k][s] = k < cnt ? nc0[s * nstride + ip] : 0.0;
      }
    }
    uint32_t headbits = 0;
    int32_t nheads = 0;
    double bmax = 0.0, amin = 1.0e308;
    double msum[K];
#pragma unroll
    for (int k = 0; k < K; ++k) msum[k] = 0.0;
#pragma unroll
    for (int k = 0; k < kWPer; ++k) {
      bv[k] = 0.0; av[k] = 1.0e308;
      if (k >= cnt) continue;
      bool head = !merge || (i0 + k) == 0;
      double pw[NS][TailDeg<NS>::D + 1], vv[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const double prev = k == 0 ? Np[s] : Nv[k > 0 ? k - 1 : 0][s];
        if ((i0 + k) > 0 && mkey(Nv[k][s]) != mkey(prev)) head = true;
        const double v = Nv[k][s] * cs[s];
        bv[k] = v > bv[k] ? v : bv[k];
        av[k] = v < av[k] ? v : av[k];
        vv[s] = v;
      }
      tail_pows<NS>(vv, pw);
      Fv[k] = Fv[k] / fs;
      if (!lds_pay) sF[i0 + k] = Fv[k];   // (payload path: sF already holds F_out by position)
      sHead[i0 + k] = head ? 1 : 0;
      if (head) { headbits |= 1u << k; ++nheads; }
      bmax = bv[k] > bmax ? bv[k] : bmax;
      amin = av[k] < amin ? av[k] : amin;
      if (window) {
#pragma unroll
        for (int m = 0; m < K; ++m) msum[m] += Fv[k] * mono_eval<NS>(M, m, pw);
      }
    }
    PROM_TS(o * 16 + 5);
    // ---- 5. combined workgroup scan (DPP): group ids (prefix sum of heads), A (prefix min of a),
    //         suffix moments; the B envelope needs no scan: records are sorted by 2^-30 buckets of
    //         b, so every later record has b_j <= b_i (1 + 2^-29) (b >= 1 only ahead of b < 1)
    const int32_t hinc = wave_prefix<int32_t>(nheads, OpAdd());
    const double ainc = wave_prefix<double>(amin, OpMin());
    double aexc = dpp_mov<0x138>(ainc);   // wave_shr:1
    if (lane == 0) aexc = 1.0e308;
    const double bw = lane_read(wave_prefix<double>(bmax, OpMax()), 63);
    if (window) {
#pragma unroll
      for (int m = 0; m < K; ++m) {
        const double inc = wave_suffix<double>(msum[m], OpAdd());
        if (lane == 0) pm_[wid][m] = inc;
        const double exc = dpp_mov<0x130>(inc);   // wave_shl:1: suffix of the later lanes
        msum[m] = lane == 63 ? 0.0 : exc;
      }
    }
    if (lane == 63) { pg_[wid] = hinc; pm_[wid][K] = ainc; }
    if (lane == 0) pm_[wid][K + 1] = bw;
    lds_barrier();
    PROM_TS(o * 16 + 6);
    int32_t gb = hinc - nheads, gtot = 0;
    double ball = 0.0;
    for (int w = 0; w < NW; ++w) {
      if (w < wid) {
        gb += pg_[w];
        aexc = pm_[w][K] < aexc ? pm_[w][K] : aexc;
      }
      if (w > wid && window) {
#pragma unroll
        for (int m = 0; m < K; ++m) msum[m] += pm_[w][m];
      }
      ball = pm_[w][K + 1] > ball ? pm_[w][K + 1] : ball;
      gtot += pg_[w];
    }
    G = gtot;
    PROM_TS(o * 16 + 3);
    // ---- 6. records, envelopes, moments (group heads), in the sorted order
    double* mo = mrecs + (int64_t)o * n_pr * ST;
    double* mm = wmom + (int64_t)o * (n_pr + 1) * K;
    {
      // forward: group ids and A
      int32_t g = gb - 1;
      double arun = aexc;
      int32_t gk[kWPer];
      double ak[kWPer];
#pragma unroll
      for (int k = 0; k < kWPer; ++k) {
        gk[k] = -1;
        ak[k] = 0.0;
        if (k >= cnt) continue;
        arun = av[k] < arun ? av[k] : arun;
        if ((headbits >> k) & 1u) { ++g; gk[k] = g; ak[k] = arun; }
      }
      PROM_TS(o * 16 + 9);
      // backward: moments
      int32_t tailB = 0;
      // histogram counts run-length encoded per thread: its keys are consecutive in the sorted order, so their
      // B and A slots are monotone and mostly shared -- one LDS atomic per run instead of one per key (lanes
      // of a wavefront hitting one slot serialise)
      int32_t runB = -1, nB = 0, runA = -1, nA = 0;
#pragma unroll
      for (int k = kWPer - 1; k >= 0; --k) {
        if (k >= cnt) continue;
        if (window && !(PROM_ORD_EXP & 8)) {
          double pw[NS][TailDeg<NS>::D + 1], vv[NS];
#pragma unroll
          for (int s = 0; s < NS; ++s) vv[s] = Nv[k][s] * cs[s];
          tail_pows<NS>(vv, pw);
#pragma unroll
          for (int m = 0; m < K; ++m) msum[m] += Fv[k] * mono_eval<NS>(M, m, pw);
        }
        if (gk[k] < 0) continue;
        const int32_t gi = gk[k];
        const int32_t i = i0 + k;
        double F = Fv[k];
        if (PROM_ORD_EXP & 1) {
        } else if (lds_pay) {
          for (int32_t j = i + 1; j < n && !sHead[j]; ++j) F += sF[(int32_t)(skey[j] & 0xffffffull)] / fs;
        } else {
          for (int32_t j = i + 1; j < n && !sHead[j]; ++j) F += sF[j];
        }
        double* r = mo + (int64_t)gi * ST;
        if (PROM_ORD_EXP & 2) {
        } else if constexpr (ST == 2) {   // one 16-byte store (lanes' records are scattered: fewer store instructions)
          *reinterpret_cast<double2*>(r) = make_double2(F, Nv[k][0]);
        } else {
          r[0] = F;
#pragma unroll
          for (int s = 0; s < NS; ++s) r[1 + s] = Nv[k][s];
        }
        if (window) {
          // later members' a are within 2^-40 of the head's: A is widened by 2^-38 to cover them
          // envelopes -> histograms over the threshold-table index (1/8 octave): slot 0 below the
          // table, slot kEnvN + 1 above it
          // (tail records, unsorted behind every candidate: B = btail covers all of them)
          // (tail records share one B slot: counted per thread and added once per wavefront below)
          const double Ag = ak[k] * (1.0 - 0x1p-38);
          if (i >= ncand) {
            ++tailB;
          } else if (!(PROM_ORD_EXP & 4)) {
            const int32_t sb = env_slot(bv[k] >= 1.0 ? ball : bv[k] * (1.0 + 0x1p-28));
            if (sb != runB) {
              if (nB) atomicAdd(&hB[runB], nB);
              runB = sb;
              nB = 0;
            }
            ++nB;
          }
          if (!(PROM_ORD_EXP & 4)) {
            const int32_t sa = env_slot(Ag);
            if (sa != runA) {
              if (nA) atomicAdd(&hA[runA], nA);
              runA = sa;
              nA = 0;
            }
            ++nA;
          }
          if (PROM_ORD_EXP & 2) {
          } else if constexpr (K % 2 == 0) {   // 16-byte stores (wmom rows are K doubles, 16-byte aligned)
            double2* mv = reinterpret_cast<double2*>(mm + (int64_t)gi * K);
#pragma unroll
            for (int m = 0; m < K; m += 2) mv[m / 2] = make_double2(M.c[m] * msum[m], M.c[m + 1] * msum[m + 1]);
          } else {
#pragma unroll
            for (int m = 0; m < K; ++m) mm[(int64_t)gi * K + m] = M.c[m] * msum[m];
          }
        }
      }
      if (nB) atomicAdd(&hB[runB], nB);
      if (nA) atomicAdd(&hA[runA], nA);
      PROM_TS(o * 16 + 10);
      {
        const int32_t tw = (int32_t)(wave_reduce_f((float)tailB, [](float a, float b) { return a + b; }) + 0.5f);
        if (lane == 0 && tw > 0) atomicAdd(&hB[env_slot(btail * (1.0 + 0x1p-28))], tw);
      }
    }
    if (window) {
      if (tid < K) {
        mm[(int64_t)G * K + tid] = 0.0;
      }
      lds_barrier();
      PROM_TS(o * 16 + 4);
      // tab_t[v] = #{g : B_g >= X_v} = sum of hB over slots >= v + 1 (and likewise tab_h from hA):
      // one workgroup suffix scan over kEnvN + 2 slots, kEnvN / kWBlock per thread
      constexpr int PT = kEnvN / kWBlock;
      int32_t cb[PT], ca_[PT], sb = 0, sa = 0;
#pragma unroll
      for (int k = PT - 1; k >= 0; --k) {
        const int32_t slot = 1 + tid * PT + k;
        sb += hB[slot]; sa += hA[slot];
        cb[k] = sb; ca_[k] = sa;
      }
      const int32_t bin = wave_suffix<int32_t>(sb, OpAdd()), ain = wave_suffix<int32_t>(sa, OpAdd());
      int32_t bex = dpp_mov<0x130>(bin), aex = dpp_mov<0x130>(ain);   // wave_shl:1
      if (lane == 63) { bex = 0; aex = 0; }
      if (lane == 0) { pi_[wid][0] = bin; pi_[wid][1] = ain; }
      lds_barrier();
      int32_t bc = bex + hB[kEnvN + 1], ac = aex + hA[kEnvN + 1];
      for (int w = NW - 1; w > wid; --w) { bc += pi_[w][0]; ac += pi_[w][1]; }
      int32_t* et = wenv + (int64_t)o * 2 * kEnvN;
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        et[tid * PT + k] = cb[k] + bc;
        et[kEnvN + tid * PT + k] = ca_[k] + ac;
      }
    }
  }
  if (tid == 0) {
    tfrac[o] = ts / fs;
    fsum[o] = fs;
    counts[o * kCnt + 0] = nact;
    counts[o * kCnt + 1] = ntr;
    counts[o * kCnt + 2] = nbl;
    counts[o * kCnt + 3] = nnf;
    counts[o * kCnt + 4] = G;
    counts[o * kCnt + 5] = sorted ? 1 : 0;
    counts[o * kCnt + 6] = (sorted && window) ? 1 : 0;
    counts[o * kCnt + 7] = dbg_word;
  }
  PROM_TS(o * 16 + 8);
}

// ---- tile windows (the planned path's step after k_order) -------------------------------------------------
// The tau window [h, t) of every (phase, 128-wavelength tile) from the phase's threshold tables (k_order,
// wenv) and the tile's Q range (tq: two halves per tile; one row per phase with orbital Doppler shift,
// else one shared row), exactly as k_tau_w would pick it for the tile's union Q range: the tile record
// {h, t, flags}; a tile whose window holds more than kHeavy records instead becomes two heavy entries, one
// per live 64-wavelength half, each with the window of its own Q range: halves of at most kChunk records go
// to the small list (one wavefront each in k_tau_p), longer ones to the big list (one workgroup each).  Two
// global counters (zeroed by k_columns8); list order is free.  A workgroup per (256 tiles, phase): the
// phase's tables are staged in LDS and its entries appended with one global atomic per list.  Its own
// kernel (not k_order's last step), so the ordering does not wait for the Doppler sigma rows.
template <int NS>
__global__ void __launch_bounds__(kBlock) k_windows(const float4* __restrict__ tq, int32_t tq_rows, int32_t n_tiles,
                                                    int64_t n_wav, const int32_t* __restrict__ counts,
                                                    const int32_t* __restrict__ wenv, int4* __restrict__ trec,
                                                    int4* __restrict__ hlist, int64_t hcap,
                                                    int32_t* __restrict__ hcnt) {
  constexpr int HCAP = 2 * kBlock;   // a workgroup's tiles give at most two entries each
  __shared__ int32_t stab[2 * kEnvN];
  __shared__ int4 hbuf[2][HCAP];
  __shared__ int32_t sHc[4];
  const int32_t o = blockIdx.y;
  const int tid = threadIdx.x;
  const int32_t tl = blockIdx.x * kBlock + tid;
  const int32_t* c = counts + o * kCnt;
  const int32_t nact = c[0], nnf = c[3], G = c[4];
  const bool sorted = c[5] != 0, wtab = c[6] != 0;
  const float4 q = tl < n_tiles ? tq[(tq_rows > 1 ? (int64_t)o * n_tiles : 0) + tl] : make_float4(0.f, 0.f, 0.f, 0.f);
  if (wtab) {
    const int32_t* et = wenv + (int64_t)o * 2 * kEnvN;
    for (int i = tid; i < 2 * kEnvN; i += kBlock) stab[i] = et[i];
  }
  if (tid < 2) sHc[tid] = 0;
  __syncthreads();
  const int32_t* hB = stab;
  const int32_t* hA = stab + kEnvN;
  const int32_t pfl = (sorted ? 1 : 0) | (nnf ? 4 : 0);
  const int32_t t_all = sorted ? G : nact;
  auto window_of = [&](float ql, float qh, int32_t* hp, int32_t* tp) {
    int32_t h = 0, t = t_all;
    if (wtab && ql >= 0.0f) {
      const int vt = env_floor((float)tail_eps<NS>() / qh * (1.0f - 0x1p-20f));
      const int vh = env_floor((float)kTauSat / ql * (1.0f + 0x1p-20f));
      t = vt > kEnvVmax ? 0 : (vt < kEnvVmin ? G : hB[vt - kEnvVmin]);
      h = vh >= kEnvVmax ? 0 : hA[vh + 1 < kEnvVmin ? 0 : vh + 1 - kEnvVmin];
    }
    *hp = h < t ? h : t;
    *tp = t;
  };
  if (tl < n_tiles) {
    const bool live1 = (int64_t)tl * kTW + 64 < n_wav;   // the second half holds wavelengths
    const bool bad = q.x < 0.0f || (live1 && q.z < 0.0f);
    const float ql = bad ? -1.0f : (live1 ? fminf(q.x, q.z) : q.x);
    const float qh = bad ? 0.0f : (live1 ? fmaxf(q.y, q.w) : q.y);
    int32_t h, t;
    window_of(ql, qh, &h, &t);
    const int32_t fl = pfl | ((wtab && t < G) ? 2 : 0);
    trec[(int64_t)o * n_tiles + tl] = make_int4(h, t, fl, 0);
    if (hlist && !nnf && t - h > kHeavy) {
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        if (hf == 1 && !live1) continue;
        int32_t hh, tt;
        window_of(hf ? q.z : q.x, hf ? q.w : q.y, &hh, &tt);
        const int32_t ff = pfl | ((wtab && tt < G) ? 2 : 0);
        const int4 e = make_int4(2 * tl + hf, hh, tt, ff | (o << 8));
        const int big = tt - hh > kChunk ? 1 : 0;
        hbuf[big][atomicAdd(&sHc[big], 1)] = e;
      }
    }
  }
  if (!hlist) return;
  __syncthreads();
  const int32_t ns = sHc[0], nb = sHc[1];
  if (tid == 0) sHc[2] = ns > 0 ? atomicAdd(&hcnt[0], ns) : 0;
  if (tid == 64) sHc[3] = nb > 0 ? atomicAdd(&hcnt[1], nb) : 0;
  __syncthreads();
  for (int32_t i = tid; i < ns; i += kBlock) hlist[sHc[2] + i] = hbuf[0][i];
  for (int32_t i = tid; i < nb; i += kBlock) hlist[hcap + sHc[3] + i] = hbuf[1][i];
}

// Fused sigma lookup -> tau -> exp(-tau) -> disk sum -> ratio.
// Grid: (wavelength tiles of kBlock, phase groups).  A thread owns one wavelength and walks the
// phases of its group: per phase it refreshes sigma_s = 10^interp(shift_o lambda) - offset (only
// when the phase's Doppler factor changed; the table bracket gallops from the previous phase's), then
// integrates the phase's chord records -- uniform across the workgroup, so scalar loads -- and writes
// R[o][w].  NS: atomic slots (0 = runtime count, sigma in LDS).  EXPK 1: table exp (the exact ocml
// path for phases flagged non-finite); 0: ocml exp everywhere (validation).
template <int NS, int EXPK>
__global__ void __launch_bounds__(kBlock) k_tau(const SigTabs4 tabv, const SigTabDev* __restrict__ tabs,
                                                const double* __restrict__ wav,
                                                const double* __restrict__ recs,
                                                const double* __restrict__ mrecs,
                                                const int32_t* __restrict__ act_ip,
                                                const double* __restrict__ fout,
                                                const int32_t* __restrict__ counts,
                                                const double* __restrict__ tfrac,
                                                const double* __restrict__ fsum, int32_t n_atoms_rt,
                                                int32_t n_pr, int32_t n_orb, int32_t phases_per_group,
                                                int64_t n_wav, const int32_t* __restrict__ wenv,
                                                const double* __restrict__ wmom,
                                                unsigned long long* __restrict__ evals,
                                                double* __restrict__ R) {
  PROM_CLK(tk0);
#ifdef PROM_TRACE
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) { g_trace[4002] = wall_clock64(); g_trace[4003] = clock64(); }
#endif
  extern __shared__ double lds[];   // EXPK 1: [2048] exp table | NS == 0: [2][n_atoms][kBlock]
  double* etab = lds;
  double* sgl = lds + (EXPK == 1 ? PROM_EXP2_TABLE_N : 0);
  if constexpr (EXPK == 1) {
    fill_exp_table(etab);
    __syncthreads();
  }
  const int64_t w = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  const bool live = w < n_wav;
  const double lam = wav[live ? w : n_wav - 1];
  const int32_t o0 = blockIdx.y * phases_per_group;
  const int32_t o1 = min(n_orb, o0 + phases_per_group);
  const int32_t ns = NS > 0 ? NS : n_atoms_rt;
  const int32_t stride = 1 + ns;
  constexpr int NR = NS > 0 ? NS : 1;
  double sg[NR];            // sigma_s at the current phase (NS > 0)
  double shv[NR];           // Doppler factor sg was computed for
#pragma unroll
  for (int s = 0; s < NR; ++s) shv[s] = __builtin_nan("");
  double* sg_l = sgl;                                  // NS == 0: [ns][kBlock]
  double* sh_l = sgl + (int64_t)ns * kBlock;           // NS == 0: [ns][kBlock]
  if constexpr (NS == 0) {
    for (int32_t s = 0; s < ns; ++s) sh_l[s * kBlock + threadIdx.x] = __builtin_nan("");
  }
  for (int32_t o = o0; o < o1; ++o) {
    PROM_CLK(tc0);
    const bool exact = !EXPK || counts[o * kCnt + 3] != 0;
    const bool sorted = !exact && counts[o * kCnt + 5] != 0;
    const bool win = sorted && counts[o * kCnt + 6] != 0;
    const int32_t n_act = counts[o * kCnt + (sorted ? 4 : 0)];
    const double* __restrict__ rec = (sorted ? mrecs : recs) + (int64_t)o * n_pr * stride;
    double acc = 0.0;
    if constexpr (NS > 0) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const double sh = tabv.t[s].shift[o];
        if (!(sh == shv[s])) {
          sg[s] = sigma_of(sh * lam, tabv.t[s]);
          shv[s] = sh;
        }
      }
      PROM_CLK(tc1);
      if (!exact) {
        double sp[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) sp[s] = sg[s] * kMinus2048OverLn2;
        int32_t i_lo = 0, i_hi = n_act;
        double q[NS];
        if (win) {
          // window [h, t) of this wavefront (see "windowed integration" above k_chords_w)
          double Q = 0.0;
#pragma unroll
          for (int s = 0; s < NS; ++s) { q[s] = sg[s] * tabv.t[s].nscale; Q += q[s] > 0.0 ? q[s] : 0.0; }
          const bool bad = !(Q <= 1.0e100);
          const float qf = (float)Q;
          float qh = qf * (1.0f + 0x1p-20f), ql = qf * (1.0f - 0x1p-20f);
          for (int off = 32; off > 0; off >>= 1) {
            qh = fmaxf(qh, __shfl_xor(qh, off, 64));
            ql = fminf(ql, __shfl_xor(ql, off, 64));
          }
          if (__ballot(bad) == 0ull) {
            const int32_t* et = wenv + (int64_t)o * 2 * kEnvN;
            const int vt = env_floor((float)tail_eps<NS>() / qh * (1.0f - 0x1p-20f));
            const int vh = env_floor((float)kTauSat / ql * (1.0f + 0x1p-20f));
            int32_t t = vt > kEnvVmax ? 0 : (vt < kEnvVmin ? n_act : et[vt - kEnvVmin]);
            int32_t h = vh >= kEnvVmax ? 0 : et[kEnvN + (vh + 1 < kEnvVmin ? 0 : vh + 1 - kEnvVmin)];
            h = h < t ? h : t;
            i_lo = __builtin_amdgcn_readfirstlane(h);
            i_hi = __builtin_amdgcn_readfirstlane(t);
          }
        }
        PROM_CLK(tc2);
        if constexpr (EXPK == 2) {
          for (int32_t i = i_lo; i < i_hi; ++i) {
            const double* r = rec + (int64_t)i * stride;
            double tau = r[1] * sg[0];
#pragma unroll
            for (int s = 1; s < NS; ++s) tau = tau + r[1 + s] * sg[s];
            acc = __builtin_fma(r[0], exp(-tau), acc);
          }
        } else {
          for (int32_t i = i_lo; i < i_hi; ++i) {
            const double* r = rec + (int64_t)i * stride;
            double y = r[1] * sp[0];
#pragma unroll
            for (int s = 1; s < NS; ++s) y = __builtin_fma(r[1 + s], sp[s], y);
            acc = acc_exp2k(acc, r[0], y, etab);
          }
        }
        PROM_CLK(tc3);
        if (win && i_hi < n_act) {
          // records [t, G): Taylor polynomial in q from the suffix moments
          const double* mp = wmom + ((int64_t)o * (n_pr + 1) + i_hi) * Monos<NS>::K;
          double mm[Monos<NS>::K];
#pragma unroll
          for (int k = 0; k < Monos<NS>::K; ++k) mm[k] = mp[k];
          acc += tail_eval<NS>(mm, q);
        }
#ifdef PROM_TRACE
        {
          const long long tc4 = clock64();
          const int64_t wv = 65536 + 8 * (((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6));
          PROM_ACC(wv + 0, tc1 - tc0);
          PROM_ACC(wv + 1, tc2 - tc1);
          PROM_ACC(wv + 2, tc3 - tc2);
          PROM_ACC(wv + 3, tc4 - tc3);
          PROM_ACC(wv + 4, 1);
          PROM_ACC(wv + 5, i_hi - i_lo);
        }
#endif
        if (evals) {
          const int nl = __popcll(__ballot(live));
          if ((threadIdx.x & 63) == 0)
            atomicAdd(&evals[(blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) & 63],
                      (unsigned long long)(i_hi - i_lo) * (unsigned long long)nl);
        }
      } else {
        const int32_t* ipl = act_ip + (int64_t)o * n_pr;
        for (int32_t i = 0; i < n_act; ++i) {
          const double* r = rec + (int64_t)i * stride;
          double tau = r[1] * sg[0];
#pragma unroll
          for (int s = 1; s < NS; ++s) tau = tau + r[1 + s] * sg[s];
          acc = acc + fout[ipl[i]] * exp(-tau);
        }
      }
    } else {
      for (int32_t s = 0; s < ns; ++s) {
        const int64_t li = (int64_t)s * kBlock + threadIdx.x;
        const double sh = tabs[s].shift[o];
        if (!(sh == sh_l[li])) {
          sg_l[li] = sigma_of(sh * lam, tabs[s]);
          sh_l[li] = sh;
        }
      }
      if (!exact && EXPK == 1) {
        for (int32_t i = 0; i < n_act; ++i) {
          const double* r = rec + (int64_t)i * stride;
          double y = r[1] * (sg_l[threadIdx.x] * kMinus2048OverLn2);
          for (int32_t s = 1; s < ns; ++s) y = __builtin_fma(r[1 + s], sg_l[s * kBlock + threadIdx.x] * kMinus2048OverLn2, y);
          acc = acc_exp2k(acc, r[0], y, etab);
        }
      } else if (!exact) {
        for (int32_t i = 0; i < n_act; ++i) {
          const double* r = rec + (int64_t)i * stride;
          double tau = r[1] * sg_l[threadIdx.x];
          for (int32_t s = 1; s < ns; ++s) tau = tau + r[1 + s] * sg_l[s * kBlock + threadIdx.x];
          acc = __builtin_fma(r[0], exp(-tau), acc);
        }
      } else {
        const int32_t* ipl = act_ip + (int64_t)o * n_pr;
        for (int32_t i = 0; i < n_act; ++i) {
          const double* r = rec + (int64_t)i * stride;
          double tau = r[1] * sg_l[threadIdx.x];
          for (int32_t s = 1; s < ns; ++s) tau = tau + r[1 + s] * sg_l[s * kBlock + threadIdx.x];
          acc = acc + fout[ipl[i]] * exp(-tau);
        }
      }
    }
    if (live) R[(int64_t)o * n_wav + w] = exact ? (acc + tfrac[o] * fsum[o]) / fsum[o] : acc + tfrac[o];
  }
#ifdef PROM_TRACE
  {
    const int64_t wv = 65536 + 8 * (((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6));
    PROM_ACC(wv + 6, clock64() - tk0);
    PROM_ACC(wv + 7, 1);
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
      g_trace[4000] = wall_clock64(); g_trace[4001] = clock64();
    }
  }
#endif
}

// ---- windowed fused kernel: sigma -> window -> exp(-tau) over [h, t) + tail polynomial -> R ------------
// A workgroup covers kTW = 128 consecutive wavelengths x kTP = 4 phases: wavefront p of the workgroup
// integrates phase o0 + p for all 128 wavelengths (2 per lane: w = tile + 64 j + lane; 128 measured
// faster than 64 or 256: wider tiles widen the union window at line cores).  Everything is
// arranged around few dependent memory round trips (about 2 us each on a busy MI355X):
//   1. wavelengths (vector loads), phase counters and Doppler factors (scalar loads);
//   2.-3. sigma_s at the shifted wavelengths: bucket directory, then a 4-node window.  UNI (no orbital
//      Doppler shift): sigma was resampled once per wavelength by the column kernel, one load;
//   4. the wavefront's window [h, t): threshold tables at its Q range (DPP max/min);
//   5. records [h, t) and the tail moments at t (scalar loads, shared by the 4 wavelengths of a lane).
constexpr int kLPT = kTW / 64;

template <int NS, bool UNI>
__global__ void __launch_bounds__(kBlock, NS <= 2 ? 6 : 4) k_tau_w(const SigTabs4 tabv, const double* __restrict__ wav,
                                                  const double* __restrict__ recs,
                                                  const double* __restrict__ mrecs,
                                                  const int32_t* __restrict__ act_ip,
                                                  const double* __restrict__ fout,
                                                  const int32_t* __restrict__ counts,
                                                  const double* __restrict__ tfrac,
                                                  const double* __restrict__ fsum, int32_t n_pr,
                                                  int32_t n_orb, int64_t n_wav,
                                                  const int32_t* __restrict__ wenv,
                                                  const double* __restrict__ wmom,
                                                  const double* __restrict__ sig,
                                                  const int4* __restrict__ trec, int32_t n_tiles,
                                                  const uint8_t* __restrict__ zfl, int32_t sig_rows,
                                                  unsigned long long* __restrict__ evals,
                                                  double* __restrict__ R) {
  constexpr int K = Monos<NS>::K;
  constexpr int ST = 1 + NS;
  __shared__ double srec[kTP][2 * 64 * ST];   // per wavefront: two chunks of 64 records
  __shared__ double sexp[1024];                // 2^(i/1024)
#ifdef PROM_TRACE
  const unsigned long long wt0 = wall_clock64();
#endif
  // the table's loads are issued with the first round of loads below and stored to LDS after them, so
  // the wave does not wait for them before issuing its other loads
  double etv[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) etv[m] = kExp2TableDev[2 * (threadIdx.x + kBlock * m)];   // kBlock == 256
  PROM_CLK(tk0);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: scalar loads below
  const int64_t tile = (int64_t)blockIdx.x * kTW;
  const int32_t o_raw = blockIdx.y * kTP + wid;
  const bool ph = o_raw < n_orb;         // this wavefront has a phase (else it mirrors the last one, unwritten)
  const int32_t o = ph ? o_raw : n_orb - 1;
  // ---- 1.
  double lam[kLPT];
  bool live[kLPT];
#pragma unroll
  for (int j = 0; j < kLPT; ++j) {
    const int64_t w = tile + 64 * j + lane;
    live[j] = w < n_wav;
    lam[j] = wav[live[j] ? w : n_wav - 1];
  }
  int4 hw = make_int4(0, 0, 0, 0);
  if constexpr (UNI) hw = trec[(int64_t)o * n_tiles + blockIdx.x];   // window chosen by k_order
  const int32_t* cp = counts + o * kCnt;
  const int32_t cA = cp[0], cG = cp[4];
  const int32_t cF = (cp[5] ? 1 : 0) | (cp[6] ? 2 : 0) | (cp[3] ? 4 : 0);
  const double tf = tfrac[o];
  // ---- 2.-3. sigma
  double sg[kLPT][NS];
  if constexpr (UNI) {
    // resampled by the trailing workgroups of k_columns8 (one row per phase with orbital Doppler shift)
    if (sig_rows > 1) {
      sig += (int64_t)o * NS * n_wav;
      if (zfl) zfl += (int64_t)o * n_wav;
    }
#pragma unroll
    for (int j = 0; j < kLPT; ++j) {
      const int64_t w = tile + 64 * j + lane;
#pragma unroll
      for (int s = 0; s < NS; ++s) sg[j][s] = sig[(int64_t)s * n_wav + (live[j] ? w : n_wav - 1)];
    }
  } else {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const double sh = tabv.t[s].shift[o];
#pragma unroll
      for (int j = 0; j < kLPT; ++j) sg[j][s] = sigma_of(sh * lam[j], tabv.t[s]);
    }
  }
  PROM_CLK(tk1);
  // ---- 4. window (q_s = sigma_s / c_s, Q = sum_s max(q_s, 0)); without orbital Doppler shift k_order
  //         has already picked it per tile
  const int32_t G = cG;
  int32_t h, t;
  if constexpr (UNI) {
    h = hw.x;
    t = hw.y;
  } else {
    bool bad = false;
    float qh = 0.0f, ql = 3.4e38f;
#pragma unroll
    for (int j = 0; j < kLPT; ++j) {
      double Qj = 0.0;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const double qs = sg[j][s] * tabv.t[s].nscale;
        Qj += qs > 0.0 ? qs : 0.0;
      }
      bad = bad || !(Qj <= 1.0e100);
      const float qf = (float)Qj;
      qh = fmaxf(qh, qf * (1.0f + 0x1p-20f));
      ql = fminf(ql, qf * (1.0f - 0x1p-20f));
    }
    for (int off = 32; off > 0; off >>= 1) {
      qh = fmaxf(qh, __shfl_xor(qh, off, 64));
      ql = fminf(ql, __shfl_xor(ql, off, 64));
    }
    bad = __ballot(bad) != 0ull;
    h = 0;
    t = (cF & 1) ? G : cA;
    if ((cF & 2) && !bad) {
      const int vt = env_floor((float)tail_eps<NS>() / qh * (1.0f - 0x1p-20f));
      const int vh = env_floor((float)kTauSat / ql * (1.0f + 0x1p-20f));
      const int32_t* et = wenv + (int64_t)o * 2 * kEnvN;
      t = vt > kEnvVmax ? 0 : (vt < kEnvVmin ? G : et[vt - kEnvVmin]);
      h = vh >= kEnvVmax ? 0 : et[kEnvN + (vh + 1 < kEnvVmin ? 0 : vh + 1 - kEnvVmin)];
    }
  }
  h = __builtin_amdgcn_readfirstlane(h < t ? h : t);
  t = __builtin_amdgcn_readfirstlane(t);
  PROM_CLK(tk2);
  // ---- 5. integrate.  Every wavefront issues its first chunk of records [h, h + 64) and the tail moments
  //         at t together (one round trip), then stores the exp table to LDS; the workgroup barrier is
  //         unconditional.
  const double* rb = ((cF & 1) ? mrecs : recs) + (int64_t)o * n_pr * ST;
  const double* mp = wmom + ((int64_t)o * (n_pr + 1) + t) * K;   // t <= G <= n_pr: the row exists
  double mm[K];
#pragma unroll
  for (int k = 0; k < K; ++k) mm[k] = mp[k];
  const double* src = rb + (int64_t)h * ST;
  const int32_t nel = (cF & 4) ? 0 : (t - h) * ST;
  double nx[ST];
#pragma unroll
  for (int c = 0; c < ST; ++c) {
    const int32_t e = 64 * c + lane;
    nx[c] = e < nel ? src[e] : 0.0;
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) sexp[threadIdx.x + kBlock * m] = etv[m];
  __syncthreads();   // sexp
  if (!ph) return;
  double acc[kLPT];
#pragma unroll
  for (int j = 0; j < kLPT; ++j) acc[j] = 0.0;
  if (cF & 4) {
    // non-finite column densities: exact reference order over the chord-order records
    const double* rb = recs + (int64_t)o * n_pr * ST;
    const int32_t* ipl = act_ip + (int64_t)o * n_pr;
    for (int32_t i = 0; i < cA; ++i) {
      const double* r = rb + (int64_t)i * ST;
      const double F = fout[ipl[i]];
#pragma unroll
      for (int j = 0; j < kLPT; ++j) {
        double tau = r[1] * sg[j][0];
#pragma unroll
        for (int s = 1; s < NS; ++s) tau = tau + r[1 + s] * sg[j][s];
        if (NS == 1 && zfl) tau = exact_tau_merged(r[1], sg[j][0], zfl, live[j] ? tile + 64 * j + lane : n_wav - 1);
        acc[j] = acc[j] + F * exp(-tau);
      }
    }
    const double fs = fsum[o];
#pragma unroll
    for (int j = 0; j < kLPT; ++j) acc[j] = (acc[j] + tf * fs) / fs;
  } else {
    const bool tail = (cF & 2) && t < G;
    // records staged through this wavefront's LDS slice in chunks of 64: one coalesced vector load per
    // chunk (the next chunk's load is in flight while this one is integrated), broadcast LDS reads
    if (h < t) {
      double sy[kLPT][NS];   // -sigma 1024/ln2: y = -tau 1024/ln2 = sum_s N_s sy_s
#pragma unroll
      for (int j = 0; j < kLPT; ++j)
#pragma unroll
        for (int s = 0; s < NS; ++s) sy[j][s] = sg[j][s] * kM1024Ln2;
      double* sr = srec[wid];
      for (int32_t c0 = 0; c0 < t - h; c0 += 64) {
        const int32_t nr = (t - h - c0) < 64 ? (t - h - c0) : 64;
        double* buf = sr + ((c0 >> 6) & 1) * 64 * ST;
#pragma unroll
        for (int c = 0; c < ST; ++c) buf[64 * c + lane] = nx[c];
        if (c0 + 64 < t - h) {
#pragma unroll
          for (int c = 0; c < ST; ++c) {
            const int32_t e = (c0 + 64) * ST + 64 * c + lane;
            nx[c] = e < nel ? src[e] : 0.0;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int32_t r = 0; r < nr; ++r) {
          const double F = buf[r * ST];
          double Nr[NS];
#pragma unroll
          for (int s = 0; s < NS; ++s) Nr[s] = buf[r * ST + 1 + s];
#pragma unroll
          for (int j = 0; j < kLPT; ++j) {
            double y = Nr[0] * sy[j][0];
#pragma unroll
            for (int s = 1; s < NS; ++s) y = __builtin_fma(Nr[s], sy[j][s], y);
            acc[j] = acc_exp1024(acc[j], F, y, sexp);
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    if (tail) {
#pragma unroll
      for (int j = 0; j < kLPT; ++j) {
        double qv[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) qv[s] = sg[j][s] * tabv.t[s].nscale;
        acc[j] += tail_eval<NS>(mm, qv);
      }
    }
#pragma unroll
    for (int j = 0; j < kLPT; ++j) acc[j] += tf;
  }
#pragma unroll
  for (int j = 0; j < kLPT; ++j)
    if (live[j]) R[(int64_t)o * n_wav + tile + 64 * j + lane] = acc[j];
  if (evals && !(cF & 4)) {
    int nl = 0;
#pragma unroll
    for (int j = 0; j < kLPT; ++j) nl += __popcll(__ballot(live[j]));
    if (lane == 0)
      atomicAdd(&evals[(blockIdx.x * kTP + wid) & 63], (unsigned long long)(t - h) * (unsigned long long)nl);
  }
#ifdef PROM_TRACE
  {
    const int64_t wv = 65536 + 8 * (((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * kTP + wid);
    const long long tk3 = clock64();
    PROM_ACC(wv + 0, tk1 - tk0);
    PROM_ACC(wv + 1, tk2 - tk1);
    PROM_ACC(wv + 2, tk3 - tk2);
    PROM_ACC(wv + 4, 1);
    PROM_ACC(wv + 5, t - h);
    PROM_ACC(wv + 6, tk3 - tk0);
    PROM_ACC(wv + 7, 1);
    // wave timeline: wall-clock start/end (100 MHz) and HW_ID | XCC_ID << 32
    const int64_t wl = 700000 + 4 * (((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * kTP + wid);
    if (lane == 0 && wl + 3 < (1 << 20)) {
      g_trace[wl] = wt0;
      g_trace[wl + 1] = wall_clock64();
      g_trace[wl + 2] = (unsigned long long)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)) |
                        ((unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) << 32);
      g_trace[wl + 3] = (unsigned long long)(t - h) * kLPT;
    }
  }
#endif
}

// ---- planned tau integration ---------------------------------------------------------------------------
// wavefronts per k_tau_p workgroup: a big heavy entry's 64-record chunks go round robin over them.  16 (one
// 1024-thread workgroup per CU at the kernel's 92 VGPRs) measured no faster than 4 on C3's heavy entries
// (17.2 against 16.1-16.4 us: half as many workgroups as big entries, so they take two each;
// profiles/r03k_bench_C3.json), so 4 stays the default
#ifndef PROM_TAU_WPG
#define PROM_TAU_WPG 4
#endif
constexpr int kTauWpg = PROM_TAU_WPG;
// k_tau_w gives every (128-wavelength tile, phase) one wavefront: the end of a run is set by the few
// windows at line cores, which hold up to ~1,000 records (Doppler-shifted multi-line spectra) against a
// median of zero.  k_tau_p instead takes k_order's plan:
//   - big entries (a 64-wavelength half tile of one phase whose window holds more than kChunk records):
//     one workgroup each; its four wavefronts take the entry's chunks of kChunk records round robin,
//     each summing its chunks in order, and the four partial sums are added in wavefront order;
//   - small entries (halves with at most kChunk records): one wavefront each;
//   - static wavefronts, one per (tile, group of 4 phases): every phase whose tile window holds at most
//     kHeavy records (nearly all wavelengths); the records of the group's phases travel as one packed load.
// Every workgroup of the grid first takes its share of the big entries (round robin), then each
// wavefront its share of the small entries, then its static unit, so long windows spread over the whole
// chip.  The result of a (phase, wavelength) depends only on its tile's and half's windows, never on the
// grid: R is identical for any sharding of the wavelength axis.
// PH: sigma has one row per phase (orbital Doppler shift), else one row for all phases.

// Records [c, c + 64) for c = 64 first, 64 (first + step), ... < n of one entry, staged through this
// wavefront's LDS slice `sr` (double buffered; `nx` holds the first chunk, already loaded), accumulated in
// order into acc: acc += F e^{-tau} at LPL wavelengths per lane.
template <int NS, int LPL>
__device__ __forceinline__ void tau_records(const double (&sy)[LPL][NS], const double* __restrict__ src, int32_t n,
                                            int32_t first, int32_t step, double (&nx)[1 + NS], int lane,
                                            double* __restrict__ sr, const double* __restrict__ sexp,
                                            double (&acc)[LPL]) {
  constexpr int ST = 1 + NS;
  const int32_t nel = n * ST;
  int32_t it = 0;
  for (int32_t c0 = 64 * first; c0 < n; c0 += 64 * step, ++it) {
    const int32_t nr = (n - c0) < 64 ? (n - c0) : 64;
    double* buf = sr + (it & 1) * 64 * ST;
#pragma unroll
    for (int c = 0; c < ST; ++c) buf[64 * c + lane] = nx[c];
    const int32_t cn = c0 + 64 * step;
    if (cn < n) {
#pragma unroll
      for (int c = 0; c < ST; ++c) {
        const int32_t e = cn * ST + 64 * c + lane;
        nx[c] = e < nel ? src[e] : 0.0;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    #pragma unroll 4
    for (int32_t r = 0; r < nr; ++r) {
      const double F = buf[r * ST];
      double Nr[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) Nr[s] = buf[r * ST + 1 + s];
#pragma unroll
      for (int j = 0; j < LPL; ++j) {
        double y = Nr[0] * sy[j][0];
#pragma unroll
        for (int s = 1; s < NS; ++s) y = __builtin_fma(Nr[s], sy[j][s], y);
        acc[j] = acc_exp1024(acc[j], F, y, sexp);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// The integration of one phase at LPL wavelengths per lane: records [h, t) (all chunks, in order), the
// tail polynomial from the moments mm, the transparent sum tf -- k_tau_w's operations in k_tau_w's order.
template <int NS, int LPL>
__device__ __forceinline__ void tau_phase(const double (&sg)[LPL][NS], const SigTabs4& tabv, const double* __restrict__ src,
                                          int32_t n, double (&nx)[1 + NS], bool tail, const double (&mm)[Monos<NS>::K], double tf,
                                          int lane, double* __restrict__ sr, const double* __restrict__ sexp,
                                          double (&acc)[LPL]) {
#pragma unroll
  for (int j = 0; j < LPL; ++j) acc[j] = 0.0;
  if (n > 0) {
    double sy[LPL][NS];
#pragma unroll
    for (int j = 0; j < LPL; ++j)
#pragma unroll
      for (int s = 0; s < NS; ++s) sy[j][s] = sg[j][s] * kM1024Ln2;
    tau_records<NS, LPL>(sy, src, n, 0, 1, nx, lane, sr, sexp, acc);
  }
  if (tail) {
#pragma unroll
    for (int j = 0; j < LPL; ++j) {
      double qv[NS];
#pragma unroll
      for (int s = 0; s < NS; ++s) qv[s] = sg[j][s] * tabv.t[s].nscale;
      acc[j] += tail_eval<NS>(mm, qv);
    }
  }
#pragma unroll
  for (int j = 0; j < LPL; ++j) acc[j] += tf;
}

template <int LPL>
__device__ __forceinline__ void tau_count(unsigned long long* __restrict__ evals, int gw, int lane, int32_t n,
                                          const bool (&live)[LPL]) {
  if (!evals) return;
  int nl = 0;
#pragma unroll
  for (int j = 0; j < LPL; ++j) nl += __popcll(__ballot(live[j]));
  if (lane == 0) atomicAdd(&evals[gw & 63], (unsigned long long)n * (unsigned long long)nl);
}

// One heavy entry {half tile, h, t, flags | phase << 8}: this lane's wavelength, its cross-sections (row of
// the entry's phase when PH), the record source, the first chunk `first` preloaded into nx.
template <int NS, bool PH>
__device__ __forceinline__ void heavy_setup(const int4 en, int32_t first, const double* __restrict__ sig,
                                            const double* __restrict__ recs, const double* __restrict__ mrecs,
                                            int32_t n_pr, int64_t n_wav, int lane, int64_t* w, bool* live,
                                            double (&sg)[1][NS], const double** src, double (&nx)[1 + NS]) {
  constexpr int ST = 1 + NS;
  const int32_t o = en.w >> 8;
  *w = (int64_t)en.x * 64 + lane;
  *live = *w < n_wav;
  {
    const double* so = sig + (PH ? (int64_t)o * NS * n_wav : 0);
#pragma unroll
    for (int s = 0; s < NS; ++s) sg[0][s] = so[(int64_t)s * n_wav + (*live ? *w : n_wav - 1)];
  }
  *src = (((en.w & 1) ? mrecs : recs)) + ((int64_t)o * n_pr + en.y) * ST;
  const int32_t nel = (en.z - en.y) * ST;
#pragma unroll
  for (int c = 0; c < ST; ++c) {
    const int32_t e = 64 * first * ST + 64 * c + lane;
    nx[c] = e < nel ? (*src)[e] : 0.0;
  }
}

// Grid: max(static units / 4, resident workgroups) workgroups of 4 wavefronts.  Static unit sw (wavefront
// blockIdx.x * 4 + wid < n_static): tile sw % n_tiles, phases 4 (sw / n_tiles) ...; round trip 1 = its
// phases' tile records {h, t, flags, tail moments} (k_order), sigma at its 128 wavelengths (2 per lane), the
// exp table; a second round trip only for the packed records of non-empty light windows.
template <int NS, bool PH, int WPG>
__global__ void __launch_bounds__(WPG * 64, WPG == 4 ? (NS <= 2 ? 5 : 3) : 1) k_tau_p(const SigTabs4 tabv, const double* __restrict__ sig,
                                                                   const double* __restrict__ recs,
                                                                   const double* __restrict__ mrecs,
                                                                   const int32_t* __restrict__ act_ip,
                                                                   const double* __restrict__ fout,
                                                                   const int32_t* __restrict__ counts,
                                                                   const double* __restrict__ tfrac,
                                                                   const double* __restrict__ fsum, int32_t n_pr,
                                                                   int32_t n_orb, int64_t n_wav,
                                                                   const double* __restrict__ wmom,
                                                                   const int4* __restrict__ trec, int32_t n_tiles,
                                                                   const int4* __restrict__ hlist, int64_t hcap,
                                                                   const int32_t* __restrict__ hcnt,
                                                                   int32_t n_static, const uint8_t* __restrict__ zfl,
                                                                   unsigned long long* __restrict__ evals,
                                                                   unsigned long long* __restrict__ tstamp,
                                                                   double* __restrict__ R) {
  constexpr int K = Monos<NS>::K;
  constexpr int ST = 1 + NS;
  constexpr int PQ = (4 * kHeavy * ST + 63) / 64;   // packed record loads per lane
  constexpr int MQ = (4 * K + 63) / 64;             // tail-moment loads per lane (four phases)
  constexpr int SR = PH ? 4 : 1;                    // sigma rows a static wavefront loads
  static_assert(4 * kHeavy * ST <= 2 * 64 * ST, "a group's packed records fit the wavefront's LDS slice");
  __shared__ double srec[WPG][2 * 64 * ST];   // per wavefront: two chunks of 64 records
  __shared__ double sexp[1024];                // 2^(i/1024)
  __shared__ double spart[WPG][64];            // big entries: the wavefronts' partial sums
#ifdef PROM_TRACE
  const unsigned long long wt0 = wall_clock64();
  long long wrk = 0;
#endif
  constexpr int NT = WPG * 64, EPT = 1024 / NT;   // threads, exp-table entries per thread
  static_assert(EPT * NT == 1024, "the exp table splits evenly over the workgroup");
  double etv[EPT];
#pragma unroll
  for (int m = 0; m < EPT; ++m) etv[m] = kExp2TableDev[2 * (threadIdx.x + NT * m)];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int32_t gw = blockIdx.x * WPG + wid;
  double* sr = srec[wid];
  // timed runs: the workgroup's first device-clock tick (the kernel's duration is the span over all)
  if (tstamp && threadIdx.x == 0) tstamp[2 * blockIdx.x] = wall_clock64();
  const int32_t nsmall = hcnt[0], nbig = hcnt[1];
  // the static unit's loads go out with the first round trip
  const int32_t sw = gw;
  const int32_t tile = sw % n_tiles, o0 = (sw / n_tiles) * 4;
  const bool has = sw < n_static && o0 < n_orb;
  const int32_t np = has ? min(4, n_orb - o0) : 0;
  // lane p < np: phase p's tile record {h, t, flags, 0}
  const int4 tv = lane < np ? trec[(int64_t)(o0 + lane) * n_tiles + tile] : make_int4(0, 0, 0, 0);
  bool live[2];
  double sg[SR][2][NS];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t w = (int64_t)tile * kTW + 64 * j + lane;
    live[j] = w < n_wav;
#pragma unroll
    for (int r = 0; r < SR; ++r) {
      const double* so = sig + (PH ? (int64_t)(o0 + r) * NS * n_wav : 0);
#pragma unroll
      for (int s = 0; s < NS; ++s) sg[r][j][s] = r < np ? so[(int64_t)s * n_wav + (live[j] ? w : n_wav - 1)] : 0.0;
    }
  }
  double tfv[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) tfv[p] = p < np ? tfrac[o0 + p] : 0.0;
#pragma unroll
  for (int m = 0; m < EPT; ++m) sexp[threadIdx.x + NT * m] = etv[m];
  __syncthreads();

  // ---- big entries: one per workgroup at a time, chunks round robin over the four wavefronts
  for (int32_t e = blockIdx.x; e < nbig; e += gridDim.x) {
    const int4 en = hlist[hcap + e];
    const int32_t h = __builtin_amdgcn_readfirstlane(en.y), t = __builtin_amdgcn_readfirstlane(en.z);
    const int32_t f4 = __builtin_amdgcn_readfirstlane(en.w);
    const int32_t o = f4 >> 8;
    int64_t w;
    bool lv;
    double sgh[1][NS], nx[ST];
    const double* src;
    heavy_setup<NS, PH>(make_int4(__builtin_amdgcn_readfirstlane(en.x), h, t, f4), wid, sig, recs, mrecs, n_pr,
                        n_wav, lane, &w, &lv, sgh, &src, nx);
    double mm[K];
    if (wid == 0 && (f4 & 2)) {
      const double* mp = wmom + ((int64_t)o * (n_pr + 1) + t) * K;   // t <= G <= n_pr: the row exists
#pragma unroll
      for (int k = 0; k < K; ++k) mm[k] = mp[k];
    }
    double sy[1][NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) sy[0][s] = sgh[0][s] * kM1024Ln2;
    double acc[1] = {0.0};
    tau_records<NS, 1>(sy, src, t - h, wid, WPG, nx, lane, sr, sexp, acc);
    int32_t nrec = 0;   // records of the chunks this wavefront took
    for (int32_t c0 = 64 * wid; c0 < t - h; c0 += 64 * WPG) nrec += min(64, t - h - c0);
    const bool lva[1] = {lv};
    tau_count<1>(evals, gw, lane, nrec, lva);
#ifdef PROM_TRACE
    wrk += nrec;
#endif
    spart[wid][lane] = acc[0];
    __syncthreads();
    if (wid == 0) {
      double r = spart[0][lane];   // the wavefronts' partial sums in order: ((p0 + p1) + p2) + ...
#pragma unroll
      for (int q = 1; q < WPG; ++q) r += spart[q][lane];
      if (f4 & 2) {
        double qv[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) qv[s] = sgh[0][s] * tabv.t[s].nscale;
        r += tail_eval<NS>(mm, qv);
      }
      r += tfrac[o];
      if (lv) R[(int64_t)o * n_wav + w] = r;
    }
    __syncthreads();
  }
  // ---- small entries: one per wavefront, first to the wavefronts of workgroups that took no big entry
  const int32_t nwv = (int32_t)gridDim.x * WPG;
  const int32_t busy = (nbig < (int32_t)gridDim.x ? nbig : (int32_t)gridDim.x) * WPG;
  for (int32_t e = (gw + nwv - busy) % nwv; e < nsmall; e += nwv) {
    const int4 en = hlist[e];
    const int32_t h = __builtin_amdgcn_readfirstlane(en.y), t = __builtin_amdgcn_readfirstlane(en.z);
    const int32_t f4 = __builtin_amdgcn_readfirstlane(en.w);
    const int32_t o = f4 >> 8;
    int64_t w;
    bool lv;
    double sgh[1][NS], nx[ST];
    const double* src;
    heavy_setup<NS, PH>(make_int4(__builtin_amdgcn_readfirstlane(en.x), h, t, f4), 0, sig, recs, mrecs, n_pr,
                        n_wav, lane, &w, &lv, sgh, &src, nx);
    const double* mp = wmom + ((int64_t)o * (n_pr + 1) + t) * K;
    double mm[K];
#pragma unroll
    for (int k = 0; k < K; ++k) mm[k] = mp[k];
    double acc[1];
    tau_phase<NS, 1>(sgh, tabv, src, t - h, nx, (f4 & 2) != 0, mm, tfrac[o], lane, sr, sexp, acc);
    const bool lva[1] = {lv};
    tau_count<1>(evals, gw, lane, t - h, lva);
#ifdef PROM_TRACE
    wrk += t - h;
#endif
    if (lv) R[(int64_t)o * n_wav + w] = acc[0];
  }
  // ---- static unit: tile, phases o0 .. o0 + np - 1
  if (np > 0) {
    int32_t h[4], t[4], fl[4], n[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      h[p] = p < np ? lane_read(tv.x, p) : 0;
      t[p] = p < np ? lane_read(tv.y, p) : 0;
      fl[p] = p < np ? lane_read(tv.z, p) : 0;
    }
    // light phases (window <= kHeavy records, not exact): packed; heavy ones are k_order's entries
    int32_t off[5];
    off[0] = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int32_t c = t[p] - h[p];
      const bool light = p < np && !(fl[p] & 4) && c <= kHeavy;
      n[p] = light ? c : -1;
      off[p + 1] = off[p] + (light ? c * ST : 0);
    }
    double pre[PQ];
#pragma unroll
    for (int q = 0; q < PQ; ++q) {
      const int32_t e = 64 * q + lane;
      pre[q] = 0.0;
      if (e < off[4]) {
        const int p = e < off[1] ? 0 : (e < off[2] ? 1 : (e < off[3] ? 2 : 3));
        const int32_t hp = p == 0 ? h[0] : (p == 1 ? h[1] : (p == 2 ? h[2] : h[3]));
        const int32_t fp = p == 0 ? fl[0] : (p == 1 ? fl[1] : (p == 2 ? fl[2] : fl[3]));
        const int32_t op = p == 0 ? off[0] : (p == 1 ? off[1] : (p == 2 ? off[2] : off[3]));
        pre[q] = ((fp & 1) ? mrecs : recs)[((int64_t)(o0 + p) * n_pr + hp) * ST + (e - op)];
      }
    }
    // element p K + k (lane e & 63 of mv[e >> 6]) holds tail moment k at phase p's window end
    double mv[MQ];
#pragma unroll
    for (int q = 0; q < MQ; ++q) {
      const int e = 64 * q + lane, p = e / K;
      const int32_t fp = p == 0 ? fl[0] : (p == 1 ? fl[1] : (p == 2 ? fl[2] : fl[3]));
      const int32_t tp = p == 0 ? t[0] : (p == 1 ? t[1] : (p == 2 ? t[2] : t[3]));
      mv[q] = (p < np && (fp & 2)) ? wmom[((int64_t)(o0 + p) * (n_pr + 1) + tp) * K + (e - p * K)] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < PQ; ++q) sr[64 * q + lane] = pre[q];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p >= np) continue;
      const int32_t o = o0 + p;
      const int r = PH ? p : 0;
      if (n[p] >= 0) {
        double sy[2][NS];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < NS; ++s) sy[j][s] = sg[r][j][s] * kM1024Ln2;
        const double* buf = sr + off[p];
        double acc[2] = {0.0, 0.0};
        #pragma unroll 4
        for (int32_t q = 0; q < n[p]; ++q) {
          const double F = buf[q * ST];
          double Nr[NS];
#pragma unroll
          for (int s = 0; s < NS; ++s) Nr[s] = buf[q * ST + 1 + s];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            double y = Nr[0] * sy[j][0];
#pragma unroll
            for (int s = 1; s < NS; ++s) y = __builtin_fma(Nr[s], sy[j][s], y);
            acc[j] = acc_exp1024(acc[j], F, y, sexp);
          }
        }
        if (fl[p] & 2) {
          double mm[K];
#pragma unroll
          for (int k = 0; k < K; ++k) mm[k] = lane_read(mv[(p * K + k) >> 6], (p * K + k) & 63);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            double qv[NS];
#pragma unroll
            for (int s = 0; s < NS; ++s) qv[s] = sg[r][j][s] * tabv.t[s].nscale;
            acc[j] += tail_eval<NS>(mm, qv);
          }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[j] += tfv[p];
          if (live[j]) R[(int64_t)o * n_wav + (int64_t)tile * kTW + 64 * j + lane] = acc[j];
        }
        tau_count<2>(evals, gw, lane, n[p], live);
#ifdef PROM_TRACE
        wrk += 2 * n[p];
#endif
      } else if (fl[p] & 4) {
        // non-finite column densities: exact reference order over the chord-order records
        const double* rb = recs + (int64_t)o * n_pr * ST;
        const int32_t* ipl = act_ip + (int64_t)o * n_pr;
        const uint8_t* zo = zfl ? zfl + (PH ? (int64_t)o * n_wav : 0) : nullptr;
        double acc[2] = {0.0, 0.0};
        for (int32_t i = 0; i < t[p]; ++i) {
          const double* rr = rb + (int64_t)i * ST;
          const double F = fout[ipl[i]];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            double tau = rr[1] * sg[r][j][0];
#pragma unroll
            for (int s = 1; s < NS; ++s) tau = tau + rr[1 + s] * sg[r][j][s];
            if (NS == 1 && zo) {
              tau = exact_tau_merged(rr[1], sg[r][j][0], zo, live[j] ? (int64_t)tile * kTW + 64 * j + lane : n_wav - 1);
            }
            acc[j] = acc[j] + F * exp(-tau);
          }
        }
        const double fs = fsum[o];
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (live[j]) R[(int64_t)o * n_wav + (int64_t)tile * kTW + 64 * j + lane] = (acc[j] + tfv[p] * fs) / fs;
      }
    }
  }
  if (tstamp) {
    __syncthreads();
    if (threadIdx.x == 0) tstamp[2 * blockIdx.x + 1] = wall_clock64();
  }
#ifdef PROM_TRACE
  {
    const int64_t wl = 700000 + 4 * (int64_t)gw;
    if (lane == 0 && wl + 3 < (1 << 20)) {
      g_trace[wl] = wt0;
      g_trace[wl + 1] = wall_clock64();
      g_trace[wl + 2] = (unsigned long long)__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)) |
                        ((unsigned long long)__builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11)) << 32);
      g_trace[wl + 3] = (unsigned long long)wrk;
    }
  }
#endif
}

// The Doppler cross-section rows of one run: polynomial rows (k_sigma_poly) when the problem's tables allow
// them (TransitDev::sig_deg), else the exp10 rows (k_sigma_rows)
static void launch_rows(hipStream_t s, TransitDev& tr, RunSlot& rs, int32_t nsig, int32_t sig_rows, bool msp,
                        hipEvent_t ev_start) {
  hipEvent_t ev_stop = nullptr;
  if (tr.kprof) {
    tr.kprof_mask |= 1u << PROM_K_SIGMA;
    ev_start = tr.kprof[2 * PROM_K_SIGMA];
    ev_stop = tr.kprof[2 * PROM_K_SIGMA + 1];
  }
  if (tr.sig_deg > 0)
    launch_sigma_poly(s, nsig, tr.sig_deg, tr.sigtab_v, tr.wav.as<double>(), tr.n_wav, sig_rows,
                      tr.sig_seg.as<prom::SigSeg>(), tr.sig_fb.as<int32_t>(), tr.n_sig_fb,
                      rs.sig.as<double>(), rs.tq.as<float4>(), msp ? 1 : 0, tr.sigtab_m.t[0].nscale,
                      rs.zfl.as<uint8_t>(), ev_start, ev_stop);
  else
    launch_sigma_rows(s, nsig, tr.sigtab_v, tr.wav.as<double>(), tr.n_wav, sig_rows, tr.sig_seg.as<prom::SigSeg>(),
                      tr.sig_fb.as<int32_t>(), tr.n_sig_fb, rs.sig.as<double>(), rs.tq.as<float4>(), msp ? 1 : 0,
                      tr.sigtab_m.t[0].nscale, rs.zfl.as<uint8_t>(), ev_start, ev_stop);
}

// prom_transit_kernel_ms: the start / stop events of kernel `id` (the given defaults when not profiling);
// kp_rec records one of them on the stream around a group of plain launches
static hipEvent_t kp_start(TransitDev& tr, int id, hipEvent_t d) {
  if (!tr.kprof) return d;
  tr.kprof_mask |= 1u << id;
  return tr.kprof[2 * id];
}
static hipEvent_t kp_stop(TransitDev& tr, int id, hipEvent_t d) { return tr.kprof ? tr.kprof[2 * id + 1] : d; }
static void kp_rec(TransitDev& tr, int id, bool stop, hipStream_t s) {
  if (!tr.kprof) return;
  tr.kprof_mask |= 1u << id;
  PROM_HIP(hipEventRecord(tr.kprof[2 * id + (stop ? 1 : 0)], s));
}

void launch_transit(hipStream_t s, TransitDev& tr, RunSlot& rs, const std::vector<AtomTable>& tables,
                    const std::vector<MolTable>& mtables, hipEvent_t* ev, int* variant, bool stage_events) {
  const int64_t per = (int64_t)tr.n_orb * tr.n_pr * tr.n_x;
  const bool wpath = tr.exp_mode && tr.n_mol == 0 && tr.n_atoms >= 1 && tr.n_atoms <= kWinMaxSpecies;
  // sigma_s(shift lambda_w) is resampled by extra workgroups of the column kernel (they run beside the
  // chord work): once per wavelength without orbital Doppler shift, once per (phase, wavelength) with it
  const bool cols8 = tr.n_mol == 0 && tr.n_x <= 64 && tr.n_terms <= 8 && tr.n_sc <= 4;
  const bool pre_sigma = cols8 && wpath && tr.window && !tr.star;
  const int32_t sig_rows = tr.uniform_shift ? 1 : tr.n_orb;
  // species merging (TransitDev::species_merge_ok) on the resampled fast path: downstream of the
  // column kernel there is one effective absorber
  const bool msp = pre_sigma && tr.species_merge_ok;
  const int32_t nsig = tr.n_atoms;                 // species the column kernel resamples
  const int32_t na = msp ? 1 : tr.n_atoms;         // species the ordering and tau kernels see
  const ColArgs& cargs = msp ? tr.colargs_m : tr.colargs;
  const int32_t n_terms = msp ? 1 : tr.n_terms;
  const double* smax = msp ? tr.sigma_max_m.as<double>() : tr.sigma_max_dev.as<double>();
  const SigTabs4& tabs4 = msp ? tr.sigtab_m : tr.sigtab_v;
  *variant = (na <= 4 ? na : 0) + (tr.exp_mode ? (wpath && tr.window ? 20 : 10) : 0);
  // stage events ride on the fast path's dispatch packets (hipExtLaunchKernelGGL start/stop events):
  // no separate event packets between the kernels
  hipEvent_t ev0 = (ev && stage_events) ? ev[0] : nullptr;   // not const: k_sigma_rows may take it
  hipEvent_t ev1 = (ev && stage_events) ? ev[1] : nullptr;
  // timed runs (no stage events): the tau kernel's interval opens at the ordering kernel's completion
  // (its stop event), not at the tau packet's own start, which the command processor stamps before the
  // packet's barrier on the ordering kernel resolves -- so it matches rocprofv3's dispatch durations
  const bool tau_fast = !(tr.n_mol > 0) && tr.exp_mode && wpath && tr.window;
  hipEvent_t ev_ord = ev ? (stage_events ? ev1 : (tau_fast ? ev[2] : nullptr)) : nullptr;
  hipEvent_t ev_tau0 = (ev && stage_events) ? ev[2] : nullptr;
  // 1. densities -> column densities -> blocking/transparency flags
  const int64_t nc = (int64_t)tr.n_orb * tr.n_pr;
  bool sig_after_order = false;   // Doppler sigma rows still to queue, after k_order (rs.sig_late)
#define PROM_COLS(SV, NSV)                                                                               \
  hipExtLaunchKernelGGL((k_columns8<SV, NSV>),                                                           \
                     dim3(col_blocks),                                                                    \
                     dim3(kBlock), 0, s, kp_start(tr, PROM_K_COLUMNS, ev0), kp_stop(tr, PROM_K_COLUMNS, nullptr), 0, \
                     cargs, n_terms,                                                                      \
                     tr.x.as<double>(), tr.n_x, tr.n_pr, tr.n_orb, tr.delta_x, tr.cy.as<double>(),        \
                     tr.cz.as<double>(), tr.body_x.as<double>(), tr.body_y.as<double>(),                   \
                     tr.planet_y.as<double>(), tr.planet_R, tr.n_moons, tr.moon_y.as<double>(),            \
                     tr.moon_R.as<double>(), smax, tr.cull_tau, rs.ncol.as<double>(),                       \
                     rs.flags.as<int32_t>(), tr.sigtab_v, tr.wav.as<double>(), tr.n_wav, rs.sig.as<double>(), \
                     pre_sigma ? rs.tq.as<float4>() : nullptr, msp ? 1 : 0, tr.sigtab_m.t[0].nscale,    \
                     (pre_sigma && tr.plan) ? rs.hcnt.as<int32_t>() : nullptr, rs.zfl.as<uint8_t>(), sig_rows, col_tcp)
#define PROM_COLS_L(NSV)                       \
  if (tr.n_x <= 8) PROM_COLS(1, NSV);          \
  else if (tr.n_x <= 16) PROM_COLS(2, NSV);    \
  else if (tr.n_x <= 32) PROM_COLS(4, NSV);    \
  else PROM_COLS(8, NSV);
  // transmission-curve path (prom_tcurve.hip, the default for one effective absorber): k_columns8, then
  // k_tc_build -> k_sigma_tc; no ordering, windows or heavy entries
  const bool tcp = tr.tcurve && cols8 && wpath && tr.window && !tr.star && na == 1 && tr.sig_seg_ok;
  TcPart* col_tcp = nullptr;   // the curves' phase partials (k_columns8 -> k_tc_build)
  if (tcp) {
    if (tr.n_pr % 32 == 0 && n_terms == 1) col_tcp = rs.tc_pp.as<TcPart>();
    tr.tc_pp_ok = col_tcp != nullptr;
    const unsigned col_blocks = (unsigned)((nc + kBlock / 8 - 1) / (kBlock / 8));
    PROM_COLS_L(0)
    PROM_HIP(hipGetLastError());
    // stats runs: {columns start, tables done, sigma start, sigma done}; timed runs: the sigma kernel's
    // interval opens at the table kernel's completion
    hipEvent_t e_tb1 = ev ? (stage_events ? ev1 : ev[2]) : nullptr;
    hipEvent_t e_sg0 = (ev && stage_events) ? ev[2] : nullptr;
    hipEvent_t e_sg1 = ev ? ev[3] : nullptr;
    const bool tw = launch_tcurve(s, tr, rs, nsig, msp, kp_start(tr, PROM_K_SIGMA_TC, e_sg0),
                                  kp_stop(tr, PROM_K_SIGMA_TC, e_sg1), kp_start(tr, PROM_K_TC_BUILD, nullptr),
                                  kp_stop(tr, PROM_K_TC_BUILD, e_tb1));
    *variant = tw ? 90 + na : 80 + na;
    return;
  }
  if (cols8) {
    // with resampling: chord workgroups padded to a multiple of 8, sigma workgroups rounded up to one
    const unsigned chord_blocks = (unsigned)((nc + kBlock / 8 - 1) / (kBlock / 8));
    // resampling workgroups: 256 wavelengths x one row each, rounded up to a multiple of 8 (XCD order)
    // orbital Doppler shift with sigma segments: the rows come from their own kernel (k_sigma_rows)
    const bool rows_seg = pre_sigma && tr.sig_seg_ok;   // (one row per phase, or one shared row without Doppler shift)
    const bool sig_fork = rows_seg && rs.aux && rs.ev_fork && rs.ev_join;
    const unsigned sig_blocks = (pre_sigma && !rows_seg) ? (((unsigned)sig_rows * grid_for(tr.n_wav) + 7u) & ~7u) : 0u;
    const unsigned col_blocks = (pre_sigma && !rows_seg) ? ((chord_blocks + 7u) & ~7u) + sig_blocks : chord_blocks;
    // the sigma rows do not depend on the columns or the ordering: with a second stream for the slot they
    // run beside k_columns8 / k_order (VALU-bound full chip beside latency-bound per-phase workgroups) and
    // join before the tile windows.  The fork point is taken before the column kernel is queued (the rows
    // wait only for the slot's previous run); PROM_SIGMA_FIRST=1 queues them before the column kernel.
    const bool sig_first = !sig_fork || (std::getenv("PROM_SIGMA_FIRST") && std::atoi(std::getenv("PROM_SIGMA_FIRST")));
    sig_after_order = rows_seg && !sig_fork && rs.sig_late && wpath;
    if (sig_fork) {
      PROM_HIP(hipEventRecord(rs.ev_fork, s));
      PROM_HIP(hipStreamWaitEvent(rs.aux, rs.ev_fork, 0));
    }
    auto sigma_rows = [&]() {
      launch_rows(sig_fork ? rs.aux : s, tr, rs, nsig, sig_rows, msp, sig_fork ? nullptr : ev0);
      if (sig_fork) PROM_HIP(hipEventRecord(rs.ev_join, rs.aux));
      else ev0 = nullptr;
    };
    if (rows_seg && sig_first && !sig_after_order) {
      sigma_rows();
    }
    // (the resampled rows always come from the row kernels: sigma segments are built for 1 to 4 species, and
    // pre_sigma implies at most kWinMaxSpecies = 4)
    PROM_REQUIRE(!pre_sigma || rows_seg, "transit: resampled rows need sigma segments");
    PROM_COLS_L(0)
    PROM_HIP(hipGetLastError());
    if (rows_seg && !sig_first) sigma_rows();
    ev0 = nullptr;
  } else {
    if (ev0) PROM_HIP(hipEventRecord(ev0, s));
    kp_rec(tr, PROM_K_COLUMNS, false, s);
    for (int32_t sc = 0; sc < tr.n_sc; ++sc) {
      const DensityDev& m = tr.dens[sc];
      const double* tab = nullptr;
      if (m.kind == PROM_DENSITY_TABULATED || m.kind == PROM_DENSITY_GRIDDED) tab = tr.tab.as<double>() + tr.tab_off[sc];
      hipLaunchKernelGGL(k_ntot, dim3(grid_for(per)), dim3(kBlock), 0, s, m, sc, tr.x.as<double>(), tr.n_x,
                         tr.cy.as<double>(), tr.cz.as<double>(), tr.n_pr, tr.n_orb, tr.body_x.as<double>(),
                         tr.body_y.as<double>(), tab, rs.ntot.as<double>());
      PROM_HIP(hipGetLastError());
    }
    double mol_max = 0.0;
    for (const auto& t : tr.terms)
      if (t.is_molecule) mol_max = std::max(mol_max, std::pow(10.0, mtables[t.table].vmax));
    if (tr.n_mol > 0) {
      hipLaunchKernelGGL(k_mol_prep, dim3(grid_for(nc * tr.n_mol, 64)), dim3(64), 0, s, tr.molslot.as<MolSlotDev>(),
                         tr.n_mol, rs.ntot.as<double>(), tr.n_x, tr.n_pr, tr.n_orb, tr.delta_x,
                         rs.mol_smp.as<double4>(), rs.mol_nin.as<int32_t>(),
                         rs.molcol.as<double>());
      PROM_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_columns, dim3(grid_for(nc, 64)), dim3(64), 0, s, tr.terms_dev.as<TermDev>(),
                       tr.n_terms, rs.ntot.as<double>(), tr.n_x, tr.n_pr, tr.n_orb, tr.delta_x,
                       tr.cy.as<double>(), tr.cz.as<double>(), tr.planet_y.as<double>(), tr.planet_R,
                       tr.n_moons, tr.moon_y.as<double>(), tr.moon_R.as<double>(),
                       tr.sigma_max_dev.as<double>(), mol_max, tr.cull_tau, rs.ncol.as<double>(),
                       rs.molcol.as<double>(), rs.flags.as<int32_t>());
    PROM_HIP(hipGetLastError());
    kp_rec(tr, PROM_K_COLUMNS, true, s);
  }
#undef PROM_COLS_L
#undef PROM_COLS
  if (tr.star) {
    // 2'. stellar spectrum: one exact chord-order kernel over the flags / columns
    if (ev1) PROM_HIP(hipEventRecord(ev1, s));
    kp_rec(tr, PROM_K_TAU, false, s);
    launch_tau_rm(s, tr, rs, na, ev);
    kp_rec(tr, PROM_K_TAU, true, s);
    *variant = 40 + (na <= 8 ? na : 0);
    PROM_HIP(hipGetLastError());
    return;
  }
  // 2. per-phase compaction, ordering, merging of equal-column chords, window tables (and, without
  //    orbital Doppler shift, every tile's window)
  const int32_t n_wtiles = (int32_t)((tr.n_wav + kTW - 1) / kTW);
  const int64_t hcap = (int64_t)tr.n_orb * 2 * n_wtiles;   // heavy entries per list: at most one per half tile
  if (wpath) {
#define PROM_CHW(NSV)                                                                                   \
  hipExtLaunchKernelGGL(k_order<NSV>, dim3(tr.n_orb), dim3(kWBlock), 0, s, kp_start(tr, PROM_K_ORDER, nullptr),    \
                     kp_stop(tr, PROM_K_ORDER, pre_sigma ? nullptr : ev_ord), 0,                           \
                     rs.flags.as<int32_t>(),                                                              \
                     tr.cfout.as<double>(), rs.ncol.as<double>(), tr.n_pr, tr.n_orb, tr.merge ? 1 : 0,   \
                     tr.window ? 1 : 0, tabs4, rs.recs.as<double>(),                                     \
                     rs.act_ip.as<int32_t>(), rs.mrecs.as<double>(), rs.counts.as<int32_t>(),            \
                     rs.tsum.as<double>(), rs.fsum.as<double>(), rs.wenv.as<int32_t>(), rs.wmom.as<double>(), \
                     btail)
    // always-tail threshold: b Q < the tail epsilon at every wavelength.  Any value keeps R exact (the
    // unsorted records' envelope is btail itself); a tight one keeps most far chords out of the sort.  The
    // factor 2^-1/4 keeps btail below every window threshold the tables can return (1/8-octave slots
    // rounded conservatively, float Q ranges widened by 2^-20), so tail records are never evaluated one by one
    const double qb = msp ? tr.qbound_m : tr.qbound_v;
    const double btail = (tr.window && qb > 0.0 && std::isfinite(qb) && !std::getenv("PROM_NO_TAIL_SPLIT"))
                             ? (na == 1 ? tail_eps<1>() : tail_eps<2>()) / qb * 0.8408964152537145 : 0.0;
    switch (na) {
      case 1: PROM_CHW(1); break;
      case 2: PROM_CHW(2); break;
      case 3: PROM_CHW(3); break;
      default: PROM_CHW(4); break;
    }
#undef PROM_CHW
    if (sig_after_order) {
      launch_rows(s, tr, rs, nsig, sig_rows, msp, nullptr);
    }
    if (pre_sigma) {
      // 2b. every tile's window from the tables and the Q ranges (after the sigma rows: join)
      if (!tr.uniform_shift && tr.sig_seg_ok && rs.aux && rs.ev_join)
        PROM_HIP(hipStreamWaitEvent(s, rs.ev_join, 0));
      const dim3 gw((unsigned)((n_wtiles + kBlock - 1) / kBlock), (unsigned)tr.n_orb);
#define PROM_WIN(NSV)                                                                                    \
  hipExtLaunchKernelGGL(k_windows<NSV>, gw, dim3(kBlock), 0, s, kp_start(tr, PROM_K_WINDOWS, nullptr),        \
                        kp_stop(tr, PROM_K_WINDOWS, ev_ord), 0, rs.tq.as<float4>(),                          \
                        sig_rows, n_wtiles, tr.n_wav, rs.counts.as<int32_t>(), rs.wenv.as<int32_t>(),       \
                        rs.trec.as<int4>(), tr.plan ? rs.hlist.as<int4>() : nullptr, hcap,                  \
                        tr.plan ? rs.hcnt.as<int32_t>() : nullptr)
      switch (na) {
        case 1: PROM_WIN(1); break;
        case 2: PROM_WIN(2); break;
        case 3: PROM_WIN(3); break;
        default: PROM_WIN(4); break;
      }
#undef PROM_WIN
    }
  } else {
    kp_rec(tr, PROM_K_ORDER, false, s);
    hipLaunchKernelGGL(k_chords, dim3(tr.n_orb), dim3(kChordBlock), 0, s, rs.flags.as<int32_t>(),
                       tr.cfout.as<double>(), rs.ncol.as<double>(), tr.n_atoms, tr.n_pr, tr.n_orb,
                       (tr.merge && tr.exp_mode && tr.n_mol == 0) ? 1 : 0, rs.recs.as<double>(), rs.act_ip.as<int32_t>(),
                       rs.mrecs.as<double>(), rs.counts.as<int32_t>(), rs.tsum.as<double>(), rs.fsum.as<double>());
    kp_rec(tr, PROM_K_ORDER, true, s);
    if (ev1) PROM_HIP(hipEventRecord(ev1, s));
  }
  PROM_HIP(hipGetLastError());
  // 3. fused sigma -> tau -> exp -> disk-sum kernel
  // phase groups: enough waves for latency hiding (~8 per SIMD over 1024 SIMDs), few enough that
  // each thread reuses its sigma bracket across several phases
  const int64_t n_tiles = (tr.n_wav + kBlock - 1) / kBlock;
  int32_t groups = (int32_t)std::max<int64_t>(1, std::min<int64_t>(tr.n_orb, (8192 + 4 * n_tiles - 1) / (4 * n_tiles)));
  const int32_t ppg = (tr.n_orb + groups - 1) / groups;
  groups = (tr.n_orb + ppg - 1) / ppg;
  dim3 g((unsigned)n_tiles, (unsigned)groups);
  const SigTabDev* tabs = tr.sigtab.as<SigTabDev>();
  const double* wav = tr.wav.as<double>();
  const double* recs = rs.recs.as<double>();
  const double* mrecs = rs.mrecs.as<double>();
  const int32_t* aip = rs.act_ip.as<int32_t>();
  const double* fo = tr.cfout.as<double>();
  const int32_t* counts = rs.counts.as<int32_t>();
  const double* tf = rs.tsum.as<double>();
  const double* fs = rs.fsum.as<double>();
  double* R = rs.R.as<double>();
#define PROM_TAU(NSV, EK)                                                                              \
  hipLaunchKernelGGL((k_tau<NSV, EK>), g, dim3(kBlock),                                                \
                     ((EK) == 1 ? PROM_EXP2_TABLE_N * sizeof(double) : 0) +                             \
                         ((NSV) == 0 ? (size_t)2 * na * kBlock * sizeof(double) : 0),                  \
                     s, tr.sigtab_v, tabs, wav, recs, mrecs, aip, fo, counts, tf, fs, na, tr.n_pr, tr.n_orb, ppg, \
                     tr.n_wav, \
                     rs.wenv.as<int32_t>(), rs.wmom.as<double>(),                                            \
                     tr.count_evals ? rs.evals.as<unsigned long long>() : nullptr, R)
#define PROM_TAU_NS(EK)                 \
  switch (na) {                         \
    case 1: PROM_TAU(1, EK); break;     \
    case 2: PROM_TAU(2, EK); break;     \
    case 3: PROM_TAU(3, EK); break;     \
    case 4: PROM_TAU(4, EK); break;     \
    default: PROM_TAU(0, EK);           \
  }
  const bool tau_w = !(tr.n_mol > 0) && tr.exp_mode && wpath && tr.window;
  if (ev && !tau_w) PROM_HIP(hipEventRecord(ev[2], s));
  if (!tau_w && tr.n_mol == 0) kp_rec(tr, PROM_K_TAU, false, s);   // (k_tau_mol: its own packet events)
  if (tr.n_mol > 0) {
    launch_tau_mol(s, tr, rs, na, g, ppg);
  } else if (tr.exp_mode && wpath && tr.window) {
#define PROM_TAUW(NSV, PMV, UV)                                                                         \
  hipExtLaunchKernelGGL((k_tau_w<NSV, UV>), dim3((unsigned)((tr.n_wav + kTW - 1) / kTW), (unsigned)((tr.n_orb + kTP - 1) / kTP)), \
                     dim3(kBlock), 0, s, kp_start(tr, PROM_K_TAU, ev_tau0), kp_stop(tr, PROM_K_TAU, ev ? ev[3] : nullptr), 0, \
                     tabs4, wav, recs, mrecs, aip, fo, counts, tf, fs, tr.n_pr,                           \
                     tr.n_orb, tr.n_wav, rs.wenv.as<int32_t>(), rs.wmom.as<double>(), rs.sig.as<double>(),  \
                     rs.trec.as<int4>(), n_wtiles, msp ? rs.zfl.as<uint8_t>() : nullptr, (UV) ? sig_rows : 1, \
                     tr.count_evals ? rs.evals.as<unsigned long long>() : nullptr, R)
#define PROM_TAUW_NS(PMV, UV)            \
  switch (na) {                          \
    case 1: PROM_TAUW(1, PMV, UV); break; \
    case 2: PROM_TAUW(2, PMV, UV); break; \
    case 3: PROM_TAUW(3, PMV, UV); break; \
    default: PROM_TAUW(4, PMV, UV); break; \
  }
    if (pre_sigma && tr.plan) {
      // planned: big and small heavy entries from k_order's lists over the whole grid, then one static
      // wavefront per (tile, 4 phases)
      const bool ph = sig_rows > 1;
      int& resident = tr.taup_resident;
      if (resident == 0) {
        int cus = 0, nb = 0;
        int dev = 0;
        PROM_HIP(hipGetDevice(&dev));
        PROM_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
#define PROM_OCC(NSV, PHV) PROM_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tau_p<NSV, PHV, kTauWpg>, kTauWpg * 64, 0))
        switch (na) {
          case 1: if (ph) { PROM_OCC(1, true); } else { PROM_OCC(1, false); } break;
          case 2: if (ph) { PROM_OCC(2, true); } else { PROM_OCC(2, false); } break;
          case 3: if (ph) { PROM_OCC(3, true); } else { PROM_OCC(3, false); } break;
          default: if (ph) { PROM_OCC(4, true); } else { PROM_OCC(4, false); } break;
        }
#undef PROM_OCC
        resident = std::max(1, cus) * std::max(1, nb);   // workgroups resident at once
      }
      const int64_t n_static = (int64_t)n_wtiles * ((tr.n_orb + 3) / 4);
      const int64_t blocks = std::max<int64_t>((n_static + kTauWpg - 1) / kTauWpg, resident);
      *variant = 30 + (na <= 4 ? na : 0);
      unsigned long long* tsp = (tr.ts_out && blocks <= tr.ts_cap) ? tr.ts_out : nullptr;
      tr.ts_blocks = tsp ? (int32_t)blocks : 0;
#define PROM_TAUP(NSV, PHV)                                                                             \
  hipExtLaunchKernelGGL((k_tau_p<NSV, PHV, kTauWpg>), dim3((unsigned)blocks), dim3(kTauWpg * 64), 0, s,   \
                        kp_start(tr, PROM_K_TAU, ev_tau0), kp_stop(tr, PROM_K_TAU, ev ? ev[3] : nullptr), 0, \
                        tabs4, rs.sig.as<double>(),                                                      \
                        recs, mrecs, aip, fo, counts, tf, fs, tr.n_pr, tr.n_orb, tr.n_wav,                \
                        rs.wmom.as<double>(), rs.trec.as<int4>(), n_wtiles, rs.hlist.as<int4>(),        \
                        hcap, rs.hcnt.as<int32_t>(), (int32_t)n_static, msp ? rs.zfl.as<uint8_t>() : nullptr, \
                        tr.count_evals ? rs.evals.as<unsigned long long>() : nullptr, tsp, R)
      switch (na) {
        case 1: if (ph) { PROM_TAUP(1, true); } else { PROM_TAUP(1, false); } break;
        case 2: if (ph) { PROM_TAUP(2, true); } else { PROM_TAUP(2, false); } break;
        case 3: if (ph) { PROM_TAUP(3, true); } else { PROM_TAUP(3, false); } break;
        default: if (ph) { PROM_TAUP(4, true); } else { PROM_TAUP(4, false); } break;
      }
#undef PROM_TAUP
    } else if (pre_sigma) { PROM_TAUW_NS(8, true) } else { PROM_TAUW_NS(2, false) }
#undef PROM_TAUW_NS
#undef PROM_TAUW
    PROM_HIP(hipGetLastError());
  }
  else if (tr.exp_mode) { PROM_TAU_NS(1) }
  else { PROM_TAU_NS(0) }
#undef PROM_TAU_NS
#undef PROM_TAU
  PROM_HIP(hipGetLastError());
  if (ev && !tau_w) PROM_HIP(hipEventRecord(ev[3], s));
  if (!tau_w && tr.n_mol == 0) kp_rec(tr, PROM_K_TAU, true, s);
}

}  // namespace prom


#ifdef PROM_TRACE
extern "C" int32_t prom_trace_read(unsigned long long* out, int32_t n, int32_t reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(prom::g_trace), sizeof(unsigned long long) * n) != hipSuccess) return -2;
  if (reset) {
    static unsigned long long z[1 << 20] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(prom::g_trace), z, sizeof(z)) != hipSuccess) return -2;
  }
  return 0;
}
#endif
