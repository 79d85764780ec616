// Molecular fused tau kernel (gasProperties.py:924-954 with MolecularConstituent.getSigmaAbs :789-818).
#include "prom_device.h"

namespace prom {

// ---- molecular fused kernel -------------------------------------------------------------------
// tau(c, w) = sum_atomic N_s sigma_s(w) + sum_mol dx * sum_x n_abs(c,x) sigma_m(P(c,x), T, lambda'_w)
// (gasProperties.py:924-954).  The slot's temperature is a constant, so the T part of the trilinear
// RegularGridInterpolator weights is folded into G once per set (k_mol_gt: g(i, w) = (1 - t_T) V[i][iT][w] +
// t_T V[i][iT + 1][w], stored times 1024 log2(10) as {g(i, w), g(i, w + 1)} pairs: 10^v = 2^(y/1024) without a
// multiply per sample).  Per thread (phase o, wavelength w) and slot the
// lambda' bracket is walked from the previous phase's; each in-table sample (P node i, weight t_P from k_mol_prep)
// then reads two 16-byte pairs, u_i = (1 - t_w) g(i, iw) + t_w g(i, iw + 1), u_{i+1} likewise, v = u_i + t_P
// (u_{i+1} - u_i), and costs 10^v and an FMA.  Out-of-table samples (P, T or lambda) take the fill value, i.e.
// sigma = 0, as in the reference (k_mol_prep compacts them away; T and lambda' are checked here).
constexpr double kLog2Ten1024 = 0x1.a934f0979a371p+11;   // 1024 log2(10)
constexpr int kMolExpN = 1024;                             // LDS exp table 2^(i/1024) (8 KB)
#ifndef PROM_MOL_WCACHE
#define PROM_MOL_WCACHE 1
#endif
constexpr bool kMolWCache = PROM_MOL_WCACHE;
#ifndef PROM_MOL_BILIN
#define PROM_MOL_BILIN 1
#endif
constexpr bool kMolBilin = PROM_MOL_BILIN;     // G as 32-byte bilinear records (else 16-byte {g, g' - g} per P node)
constexpr uint32_t kMolRec = kMolBilin ? 32u : 16u;
// k_tau_mol (one molecular slot, table exp): the G records of the workgroup's lambda' node range, all P intervals,
// staged in LDS (double2 units; 19 KB: with the 8 KB exp table and 4 KB of bracket nodes, 5 workgroups per CU)
constexpr int kMolStageD2 = 1216;
constexpr int kMolStageMargin = 1;
#ifndef PROM_MOL_MTOL
#define PROM_MOL_MTOL 40
#endif
constexpr double kMolMirrorTol = 1.0 / (double)(1ull << PROM_MOL_MTOL);
#ifndef PROM_MOL_STAGE
#define PROM_MOL_STAGE 1
#endif
struct OpMinI { __device__ int32_t operator()(int32_t a, int32_t b) const { return a < b ? a : b; } };
struct OpMaxI { __device__ int32_t operator()(int32_t a, int32_t b) const { return a > b ? a : b; } };   // k_tau_mol keeps each lane's lambda' bracket nodes in LDS
constexpr int32_t kMolLast = 1 << 30;    // list entry flags (k_mol_list): the record's last entry (.w = its weight)
constexpr int32_t kMolEmpty = 1 << 29;   //   the zero-weight entry of a record without in-table samples

// 2^(y/1024) - w = 2^(k >> 10) T[k & 1023] exp(e) - w, k = rint(y), e = (y - k) ln2/1024 in [-ln2/2048, ln2/2048],
// exp(e) by its cubic Taylor polynomial in e (truncation e^4/24 <= 5.5e-16 relative; acc_exp1024's arithmetic
// without the accumulation).  Horner in e rather than in y - k: the inner coefficients 1/2 and 1 are inline
// constants, so no FMA needs two non-inline constants (4 operations for the polynomial instead of 5)
constexpr double kLn2Over1024 = 0x1.62e42fefa39efp-11;
__device__ __forceinline__ double exp2_1024_minus(double y, const double* __restrict__ tab, double w) {
  const double k = __builtin_rint(y);
  const int ki = (int)k;
  const double e = (y - k) * kLn2Over1024;
  double p = __builtin_fma(e, 1.0 / 6.0, 0.5);
  p = __builtin_fma(e, p, 1.0);
  p = __builtin_fma(e, p, 1.0);
  return __builtin_fma(__builtin_amdgcn_ldexp(tab[ki & (kMolExpN - 1)], ki >> 10), p, -w);
}

// acc + F exp(-tau), y = -tau 1024/ln2, with exp2_1024_minus's polynomial (acc_exp1024 keeps the Horner form in
// y - k: the windowed tau kernels' register allocation is tuned to it)
__device__ __forceinline__ double acc_exp1024_e(double acc, double F, double y, const double* __restrict__ tab) {
  const double k = __builtin_rint(y);
  const int ki = (int)k;
  const double e = (y - k) * kLn2Over1024;
  double p = __builtin_fma(e, 1.0 / 6.0, 0.5);
  p = __builtin_fma(e, p, 1.0);
  p = __builtin_fma(e, p, 1.0);
  return __builtin_fma(F * __builtin_amdgcn_ldexp(tab[ki & (kMolExpN - 1)], ki >> 10), p, acc);
}

// G of one slot: per P interval i in [0, n_p - 2] and lambda' interval w, 32 bytes {g_i, s_i, g_{i+1} - g_i,
// s_{i+1} - s_i} with g_i = g(i, w), s_i = g(i, w + 1) - g(i, w), at the slot's T (unused when T is outside the
// table), so a sample's bilinear value g_i + t_w s_i + t_p ((g_{i+1} - g_i) + t_w (s_{i+1} - s_i)) is three FMAs
// from one 32-byte record (two 16-byte loads)
__global__ void k_mol_gt(const double* __restrict__ Tg, int32_t n_t, double T, const double* __restrict__ V,
                         int32_t n_p, int64_t n_w, double2* __restrict__ G) {
  int64_t it = 0;
  double tt = 0.0;
  if (!rgi_bracket(Tg, n_t, T, &it, &tt)) return;
  const int64_t nw1 = n_w - 1;
  const int64_t tot = (int64_t)(kMolBilin ? max(n_p - 1, 1) : n_p) * nw1;
  // stored as y = 1024 log2(10) v (the lookups' exponent scale: 10^v = 2^(y/1024), no multiply per sample)
  auto y = [&](int64_t i, int64_t w) {
    const double* v0 = V + (i * n_t + it) * n_w + w;
    return ((1.0 - tt) * v0[0] + tt * v0[n_w]) * kLog2Ten1024;
  };
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < tot; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = k / nw1, w = k - i * nw1;
    if (!kMolBilin) {
      const double g0 = y(i, w);
      G[k] = make_double2(g0, y(i, w + 1) - g0);
      continue;
    }
    const int64_t i1 = min<int64_t>(i + 1, n_p - 1);
    const double g0 = y(i, w), s0 = y(i, w + 1) - g0;
    const double g1 = y(i1, w), s1 = y(i1, w + 1) - g1;
    G[2 * k] = make_double2(g0, s0);
    G[2 * k + 1] = make_double2(g1 - g0, s1 - s0);
  }
}

void launch_mol_gt(hipStream_t s, const MolSlotDev& md) {
  const int64_t tot = (int64_t)(kMolBilin ? std::max(md.n_p - 1, 1) : md.n_p) * (md.n_w - 1);
  const unsigned nb = (unsigned)std::min<int64_t>((tot + kBlock - 1) / kBlock, 8192);
  hipLaunchKernelGGL(k_mol_gt, dim3(nb), dim3(kBlock), 0, s, md.T, md.n_t, md.temp, md.V, md.n_p, md.n_w,
                     const_cast<double2*>(md.G));
  PROM_HIP(hipGetLastError());
}

template <int NSA, int EXPK, bool M1>
__global__ void __launch_bounds__(kBlock) k_tau_mol(const SigTabs4 tabv, const MolSlotDev* __restrict__ ms,
                                                    int32_t n_mol, int64_t lst_stride,
                                                    const double* __restrict__ wav,
                                                    const double* __restrict__ recs,
                                                    const int32_t* __restrict__ act_ip,
                                                    const double* __restrict__ fout,
                                                    const int32_t* __restrict__ counts,
                                                    const double* __restrict__ tfrac,
                                                    const double* __restrict__ fsum, int32_t n_pr,
                                                    int32_t n_orb, int32_t phases_per_group, int64_t n_wav,
                                                    double delta_x, const double4* __restrict__ lst,
                                                    const int32_t* __restrict__ rend, double* __restrict__ R,
                                                    unsigned long long* __restrict__ evals, int32_t stage) {
  __shared__ double etab[kMolExpN];   // exp table 2^(i/1024)
  // (with the LDS stage the table is filled in the stage's load round and barrier, below)
  const bool etab_late = M1 && EXPK && kMolBilin && PROM_MOL_STAGE && stage != 0;
  if (EXPK && !etab_late) {
    for (int i = threadIdx.x; i < kMolExpN; i += kBlock) etab[i] = kExp2TableDev[i * (PROM_EXP2_TABLE_N / kMolExpN)];
    __syncthreads();
  }
  const int64_t w = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  const bool live = w < n_wav;
  const double lam = wav[live ? w : n_wav - 1];
  const int32_t o0 = blockIdx.y * phases_per_group;
  const int32_t o1 = min(n_orb, o0 + phases_per_group);
  constexpr int ST = 1 + NSA;
  constexpr int NR = NSA > 0 ? NSA : 1;
  double sg[NR], shv[NR];
#pragma unroll
  for (int s = 0; s < NR; ++s) { shv[s] = __builtin_nan(""); sg[s] = 0.0; }
  unsigned long long npow = 0;   // stats runs: this lane's 10^v evaluations (in-table samples)

  // per slot (at most 4): T inside its table (uniform), the lambda' bracket (iw, t_w) of the current phase, the
  // in-table bit, and the walk's start
  uint32_t tin = 0;
  __amdgpu_buffer_rsrc_t rsv[M1 ? 1 : 4];   // each slot's G as one buffer (< 2^31 bytes: the launcher checks)
  uint32_t rowbv[M1 ? 1 : 4];               // bytes per G row
  double offv[M1 ? 1 : 4];                  // each slot's offset (10^v - offset)
#pragma unroll
  for (int m = 0; m < (M1 ? 1 : 4); ++m) {
    const bool valid = m < n_mol;   // (unused slots: empty buffers, never selected)
    offv[m] = valid ? ms[m].offset : 0.0;
    int64_t it;
    double tt;
    if (valid && rgi_bracket(ms[m].T, ms[m].n_t, ms[m].temp, &it, &tt)) tin |= 1u << m;
    rowbv[m] = valid ? (uint32_t)(ms[m].n_w - 1) * kMolRec : 0u;
    rsv[m] = __builtin_amdgcn_make_buffer_rsrc(valid ? const_cast<double2*>(ms[m].G) : nullptr, (short)0,
                                               valid ? (int)((uint32_t)(kMolBilin ? max(ms[m].n_p - 1, 1) : ms[m].n_p) * rowbv[m]) : 0,
                                               0x00020000);
  }
  double shp[M1 ? 1 : 4];   // each slot's Doppler factor at the previous phase (uniform)
#pragma unroll
  for (int m = 0; m < (M1 ? 1 : 4); ++m) shp[m] = __builtin_nan("");
  int64_t iwv[4] = {-1, -1, -1, -1};
  double twv[4] = {0.0, 0.0, 0.0, 0.0};
  // the lane's current bracket nodes {W[h], W[h + 1]} per slot (a phase whose lambda' stays inside them reuses h
  // with no load), and each slot's table ends (uniform, read once)
  // (in LDS, the lane's own column: registers would cost a wave per SIMD)
  __shared__ double2 wbr[M1 ? 1 : 4][kBlock];
  uint32_t inb = 0;
  // Staging (one slot, table exp): every sample of a phase reads G records of the same P intervals at the lanes'
  // lambda' nodes, and a workgroup's 256 wavelengths cover a few tens of nodes at most (C5: ~6-27), so the records
  // of [st_lo, st_lo + st_n) x all intervals are copied to LDS once and the samples read them there: one 32-byte LDS
  // read pair per sample instead of two vector-L1 loads (the L1's 64 bytes per clock per CU bound the global
  // variant, profiles/r05y_*).  Staged once, at the group's first phase; a later phase whose node range leaves the
  // staged one (rarely: the Doppler factors move lambda' by ~1e-6), or a range too wide for the buffer, reads those
  // records from global memory for that phase.
  constexpr bool STG = M1 && EXPK && kMolBilin && PROM_MOL_STAGE;
  __shared__ double2 gst[STG ? kMolStageD2 : 1];
  __shared__ int32_t red[2][kBlock / 64];
  int32_t st_lo = 0, st_n = 0;
  bool st_done = stage == 0;   // (PROM_MOL_STAGE=0: every sample reads global memory)
  bool wasc = false;   // the wave's wavelengths ascending (lane order)
  if constexpr (STG) {
    const double prev = __shfl_up(lam, 1);
    wasc = __ballot((threadIdx.x & 63) > 0 && !(lam >= prev)) == 0ull;
  }
  const int32_t n_int = M1 ? max(ms[0].n_p - 1, 1) : 0;
  for (int32_t o = o0; o < o1; ++o) {
    const bool exact = !EXPK || counts[o * kCnt + 3] != 0;
    const int32_t n_act = counts[o * kCnt + 0];
    const double* __restrict__ rec = recs + (int64_t)o * n_pr * ST;
#pragma unroll
    for (int s = 0; s < NSA; ++s) {
      const double sh = tabv.t[s].shift[o];
      if (!(sh == shv[s])) {
        sg[s] = sigma_of(sh * lam, tabv.t[s]);
        shv[s] = sh;
      }
    }
#pragma unroll
    for (int m = 0; m < (M1 ? 1 : 4); ++m) {
      if (m >= n_mol) break;
      const double* __restrict__ W = ms[m].W;
      const int64_t nw = ms[m].n_w;
      // the previous phase's Doppler factor (no orbital Doppler shift: every phase's): the same bracket, weight
      // and in-table bit, nothing to do
      const double sh = ms[m].shift[o];
      if (sh == shp[m]) continue;
      shp[m] = sh;
      const double lw = sh * lam;
      // scipy: i = searchsorted(W, lw, 'left') - 1 clipped to [0, n-2], fill outside [W[0], W[n-1]]
      const bool ok = ((tin >> m) & 1u) && lw >= W[0] && lw <= W[nw - 1];
      inb = ok ? (inb | (1u << m)) : (inb & ~(1u << m));
      if (!ok) continue;
      int64_t h = iwv[m];
      double2 wb = kMolWCache && h >= 0 ? wbr[m][threadIdx.x] : make_double2(0.0, 0.0);
      // W[h] < lambda' <= W[h + 1] (the common case: adjacent phases' Doppler factors differ by ~1e-6): h stays,
      // no load; otherwise search (first phase) or walk from the previous phase's bracket
      if (!kMolWCache || h < 0 || !(wb.x < lw && lw <= wb.y)) {
        if (h < 0) {
          // first phase: the linear guess on the node range, kept when it is scipy's bracket (uniform grids, e.g.
          // ExoMol's bin edges: two loads instead of a ~16-load dependent bisection), else bisection
          const double W0 = W[0], WN = W[nw - 1];
          int64_t g = (int64_t)((lw - W0) * ((double)(nw - 1) / (WN - W0)));
          g = g < 0 ? 0 : (g > nw - 2 ? nw - 2 : g);
          if (W[g] < lw && lw <= W[g + 1]) {
            h = g;
          } else {
            int64_t lo = 0, hi = nw - 1;
            while (hi - lo > 1) {
              const int64_t mid = (lo + hi) >> 1;
              if (W[mid] < lw) lo = mid; else hi = mid;
            }
            h = lo;
          }
        } else {
          while (h < nw - 2 && W[h + 1] < lw) ++h;
          while (h > 0 && !(W[h] < lw)) --h;
        }
        iwv[m] = h;
        wb = make_double2(W[h], W[h + 1]);
        if (kMolWCache) wbr[m][threadIdx.x] = wb;
      }
      twv[m] = (lw - wb.x) / (wb.y - wb.x);
    }
    const int32_t* ipl = act_ip + (int64_t)o * n_pr;
    double acc = 0.0;
    // The phase's in-table samples are one flat list in record order (k_mol_list: {P weight, n_abs, flags | slot
    // << 16 | P bracket, record weight}), every record at least one entry (a zero-weight one if it has no in-table
    // sample), its last entry flagged kMolLast and carrying the record's weight.  Read with wave-uniform scalar
    // loads four at a time: the four samples' G reads, 10^v and products are independent; then they are added into
    // the current record's sum, the flagged ones finishing their record (e^-tau) -- no record-end table, no scalar
    // round trip per record.  Per sample n_abs (10^v - offset), the reference's order of the subtraction
    // (gasProperties.py:811-818, 10**interp - offset).
    const double4* __restrict__ lo = lst + (int64_t)o * lst_stride;
    const int32_t K = n_act > 0 ? rend[(int64_t)o * n_pr + n_act - 1] : 0;
    // per slot: the lane's byte offset of its lambda' pair in a G row and the in-table mask (1 / 0: a product, no
    // select; out-of-table lanes read the row's first pair, finite)
    uint32_t boff[M1 ? 1 : 4];
    double msk[M1 ? 1 : 4];
#pragma unroll
    for (int m = 0; m < (M1 ? 1 : 4); ++m) {
      const bool in = ((inb >> m) & 1u) != 0;
      boff[m] = in ? (uint32_t)iwv[m] * kMolRec : 0u;
      msk[m] = in ? 1.0 : 0.0;
    }
    const double ydx = (M1 ? msk[0] : 1.0) * (delta_x * kM1024Ln2);
    bool use_st = false;
    uint32_t ldso = 0, srow = 0;   // the lane's byte offset in a staged row, the staged row's bytes
    if constexpr (STG) {
      if (!exact) {
        // the wave's lambda' node range [mn, mx] over its in-table lanes: with ascending wavelengths (the common
        // case, checked once per wave) the first and last in-table lanes hold it; otherwise a wave reduction
        const bool in0 = (inb & 1u) != 0;
        const int32_t iw = (int32_t)iwv[0];
        const unsigned long long bal = __ballot(in0);
        int32_t mn = 0x7fffffff, mx = -1;
        if (bal != 0ull) {
          if (wasc) {
            mn = __builtin_amdgcn_readlane(iw, __builtin_ctzll(bal));
            mx = __builtin_amdgcn_readlane(iw, 63 - __builtin_clzll(bal));
          } else {
            mn = lane_read(wave_prefix<int32_t>(in0 ? iw : 0x7fffffff, OpMinI()), 63);
            mx = lane_read(wave_prefix<int32_t>(in0 ? iw : -1, OpMaxI()), 63);
          }
        }
        if (!st_done) {
          // the group's first table-exp phase stages the workgroup's range with a margin of kMolStageMargin nodes
          // each side (later phases' ranges stay inside it unless lambda' moves that far; a wave whose range leaves
          // it reads that phase's records from global memory)
          const int wid = threadIdx.x >> 6;
          double et[kMolExpN / kBlock];   // (the exp table's loads in flight across the range exchange)
#pragma unroll
          for (int j = 0; j < kMolExpN / kBlock; ++j)
            et[j] = kExp2TableDev[(threadIdx.x + j * kBlock) * (PROM_EXP2_TABLE_N / kMolExpN)];
          if ((threadIdx.x & 63) == 0) { red[0][wid] = mn; red[1][wid] = mx; }
          __syncthreads();
          int32_t gmn = 0x7fffffff, gmx = -1;
#pragma unroll
          for (int v = 0; v < kBlock / 64; ++v) { gmn = min(gmn, red[0][v]); gmx = max(gmx, red[1][v]); }
          gmn = __builtin_amdgcn_readfirstlane(gmn);   // (uniform: scalar registers for the stage's bounds)
          gmx = __builtin_amdgcn_readfirstlane(gmx);
          if (gmn <= gmx) {
            const int32_t nw1 = (int32_t)(ms[0].n_w - 1);
            const int32_t lo_ = max(0, gmn - kMolStageMargin), hi_ = min(nw1 - 1, gmx + kMolStageMargin);
            const int32_t n_ = hi_ - lo_ + 1;
            if (n_ * n_int * 2 <= kMolStageD2) {
              const double2* __restrict__ G = ms[0].G;
              for (int e = threadIdx.x; e < n_int * n_ * 2; e += kBlock) {
                const int i = e / (2 * n_), rr = e - i * 2 * n_;
                gst[e] = G[2 * ((int64_t)i * nw1 + lo_) + rr];
              }
              st_lo = lo_;
              st_n = n_;
            }
          }
#pragma unroll
          for (int j = 0; j < kMolExpN / kBlock; ++j) etab[threadIdx.x + j * kBlock] = et[j];
          __syncthreads();
          st_done = true;
        }
        use_st = st_n > 0 && (mn > mx || (st_lo <= mn && mx < st_lo + st_n));
        if (use_st) {
          ldso = (in0 ? (uint32_t)(iw - st_lo) : 0u) * kMolRec;
          srow = __builtin_amdgcn_readfirstlane((uint32_t)st_n * kMolRec);
        }
      }
    }
    int32_t nsl[4] = {0, 0, 0, 0};   // samples per slot (uniform; stats)
    // one instance per exp mode (uniform per phase), so the four samples' loads issue together
    auto samples = [&](auto ex, auto lm) {
      constexpr bool EX = decltype(ex)::value;
      constexpr bool LM = decltype(lm)::value;   // records from the LDS stage
      int32_t r = 0;
      double sm = 0.0;
      if constexpr (!EX && NSA == 0) acc = lo[K].w;   // the weight sum of the records k_mol_list folded (e^0)
      auto finish = [&](double F) {
        if constexpr (!EX && NSA == 0) {
          // -tau 1024/ln2 = sm (mask delta_x (-1024/ln2)), the factor per phase
          acc = acc_exp1024_e(acc, F, sm * ydx, etab);
          sm = 0.0;
          ++r;
          return;
        }
        const double tm = (!EX && M1 ? sm * msk[0] : sm) * delta_x;
        double tau = NSA == 0 ? tm : 0.0;
        if constexpr (NSA > 0) {
          const double* rr = rec + (int64_t)r * ST;
#pragma unroll
          for (int s = 0; s < NSA; ++s) tau = tau + rr[1 + s] * sg[s];
          tau = tau + tm;
        }
        sm = 0.0;
        if constexpr (!EX) acc = acc_exp1024_e(acc, F, tau * kM1024Ln2, etab);
        else acc = acc + fout[ipl[r]] * exp(-tau);
        ++r;
      };
      // batches of NB samples from k0 (the ocml exp10 path: one sample at a time, few registers)
      auto batch = [&](auto nbc, int32_t k0) {
        constexpr int NB = decltype(nbc)::value;
        static_assert(NB <= kMolListPad, "k_mol_list pads each phase's list by kMolListPad entries");
        struct Qb { double4 q[NB]; };
        // the batch's entries in one scalar read (k_mol_list pads each phase's list with valid zero-weight
        // entries: any past K are looked up and not added)
        const Qb qb = *reinterpret_cast<const Qb*>(lo + k0);
        double c[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const double4 q = qb.q[j];
          const int32_t code = (int32_t)__double_as_longlong(q.z);   // (integer bits: scalar decode)
          const int32_t m = M1 ? 0 : (code >> 16) & 3, pi = code & 0xffff;
          // the slot's bracket (m uniform: selects, no indexing of the register arrays)
          uint32_t bo = boff[0];
          double tw = twv[0], mk = msk[0], off = offv[0];
          __amdgpu_buffer_rsrc_t rs = rsv[0];
          uint32_t rowb = rowbv[0];
          if constexpr (!M1) {
#pragma unroll
            for (int mm = 1; mm < 4; ++mm)
              if (m == mm) { bo = boff[mm]; tw = twv[mm]; mk = msk[mm]; off = offv[mm]; rs = rsv[mm]; rowb = rowbv[mm]; }
          }
          // P interval pi's record at the lane's lambda' (k_mol_gt): two buffer loads, the row at a uniform offset
          // (soffset), the lane's record at its own
          const uint32_t so = (uint32_t)pi * rowb;
          double2 ga, gb;
          if constexpr (LM) {
            const double2* sp = reinterpret_cast<const double2*>(reinterpret_cast<const char*>(gst) +
                                                                 ((uint32_t)pi * srow + ldso));
            ga = sp[0];
            gb = sp[1];
          } else {
            ga = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, bo, so, 0));
            // (PROM_MOL_BILIN=0: rows pi and pi + 1, {g, g' - g} each)
            gb = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, kMolBilin ? bo + 16 : bo,
                                                                                   kMolBilin ? so : so + rowb, 0));
          }
          double v;
          if constexpr (kMolBilin) {
            v = __builtin_fma(q.x, __builtin_fma(tw, gb.y, gb.x), __builtin_fma(tw, ga.y, ga.x));
          } else {
            const double a = __builtin_fma(tw, ga.y, ga.x), b = __builtin_fma(tw, gb.y, gb.x);
            v = __builtin_fma(q.x, b - a, a);
          }
          if constexpr (!EX) {
            // 10^v - offset, 10^v = 2^(y/1024), y = v 1024 log2(10), from the LDS table (relative error ~ |v| ln10
            // 2^-53 from the argument, ~6e-15 at the table's floor); n_abs (10^v - offset) is added by one FMA
            // below, the in-table mask applied to the record's sum (one slot) or here (several)
            const double e = exp2_1024_minus(v, etab, off);
            c[j] = M1 ? e : e * mk;
          } else {
            // (v is 1024 log2(10) times the table value: 2^(v/1024) = 10^value.  The scaling of G, k_mol_gt, adds
            // |value| ln10 2^-53 relative per sample (8e-15 at -30) next to ocml's exp2; the validation test
            // test_transit_ocml_exp_mode checks this path against the reference's golden R at 1e-12)
            const double e = exp2(v * 0x1p-10);
            c[j] = (q.y * (e - off)) * mk;
          }
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if (k0 + j >= K) break;
          const int32_t code = (int32_t)__double_as_longlong(qb.q[j].z);
          if constexpr (!EX) sm = __builtin_fma(qb.q[j].y, c[j], sm);
          else sm += c[j];
          if (code & kMolLast) finish(qb.q[j].w);
        }
      };
      if constexpr (EX) {
        for (int32_t k0 = 0; k0 < K; ++k0) batch(std::integral_constant<int, 1>{}, k0);
      } else {
        // fours, then a pair and a single for the phase's last K mod 4 (no lookups past K)
        int32_t k0 = 0;
        for (; k0 + 4 <= K; k0 += 4) batch(std::integral_constant<int, 4>{}, k0);
        if (K - k0 >= 2) {
          batch(std::integral_constant<int, 2>{}, k0);
          k0 += 2;
        }
        if (k0 < K) batch(std::integral_constant<int, 1>{}, k0);
      }
    };
    if (!EXPK || exact) samples(std::true_type{}, std::false_type{});
    else if (STG && use_st) samples(std::false_type{}, std::true_type{});
    else samples(std::false_type{}, std::false_type{});
    if (evals) {
      // (stats runs: the phase's listed samples per slot, the zero-weight entries of empty records excluded)
      for (int32_t k = 0; k < K; ++k) {
        const int32_t code = (int32_t)__double_as_longlong(lo[k].z);
        if (!(code & kMolEmpty)) nsl[(code >> 16) & 3] += 1;
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) npow += ((inb >> m) & 1u) ? (unsigned long long)nsl[m] : 0ull;
    }
    if (live) R[(int64_t)o * n_wav + w] = exact ? (acc + tfrac[o] * fsum[o]) / fsum[o] : acc + tfrac[o];
  }
  if (evals && live && npow) atomicAdd(&evals[(blockIdx.x * 4 + (threadIdx.x >> 6)) & 63], npow);
}

// Per phase: the in-table samples of its records (k_chords' active chords, chord order) as one flat list for
// k_tau_mol: record r's samples of every molecular slot (k_mol_prep's compacted rows) at [rend[r - 1], rend[r]),
// each {P weight, n_abs, flags | slot << 16 | P bracket, 0}; a record without in-table samples gets one zero-weight
// entry (kMolEmpty), and each record's last entry is flagged kMolLast with .w = the record's weight (recs[.][0]).
// kMolListPad valid zero-weight entries follow the list.  One workgroup per phase.
__global__ void __launch_bounds__(kBlock) k_mol_list(const MolSlotDev* __restrict__ ms, int32_t n_mol,
                                                     const int32_t* __restrict__ counts,
                                                     const int32_t* __restrict__ act_ip,
                                                     const double4* __restrict__ msmp,
                                                     const int32_t* __restrict__ mnin,
                                                     const double* __restrict__ recs, int32_t n_st, int32_t n_pr,
                                                     int32_t n_orb, int32_t n_x, int64_t lst_stride,
                                                     int32_t fold_empty, const int32_t* __restrict__ mirror,
                                                     double4* __restrict__ lst, int32_t* __restrict__ rend) {
  __shared__ int32_t wsum[kBlock / 64];
  __shared__ double wfe[kBlock / 64];
  __shared__ int32_t rmap[kMolMirrorMax];   // chord -> this phase's record (mirror merging)
  const int32_t o = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int32_t n_act = counts[o * kCnt];
  // (table-exp phases without atomic species: a record without in-table samples adds exactly its weight, e^0 --
  // summed here instead of listed)
  const bool fold = fold_empty && counts[o * kCnt + 3] == 0;
  const int64_t nc = (int64_t)n_orb * n_pr;
  double4* lo = lst + (int64_t)o * lst_stride;
  // Mirror merging (folded phases, mirror != null: the launcher passes it for n_pr <= kMolMirrorMax): chord ip and
  // its mirror image mirror[ip] (z -> -z, paired on the host) see the same densities about a body on the y axis, so
  // when both are active records with equal sample lists -- every slot's in-table count, P brackets equal, P
  // weights and n_abs within kMolMirrorTol (relative) -- their tau agree to ~2^-42 and the pair is integrated once,
  // by the lower record with the summed weight (the bound of k_chords' column merging, R moves by < 1e-13)
  const bool mrg = fold && mirror != nullptr;
  if (mrg) {
    for (int32_t ip = tid; ip < n_pr; ip += kBlock) rmap[ip] = -1;
    __syncthreads();
    for (int32_t r = tid; r < n_act; r += kBlock) rmap[act_ip[(int64_t)o * n_pr + r]] = r;
    __syncthreads();
  }
  int32_t base = 0;
  double fe_sum = 0.0;
  for (int32_t r0 = 0; r0 < n_act; r0 += kBlock) {
    const int32_t r = r0 + tid;
    const int32_t ip = r < n_act ? act_ip[(int64_t)o * n_pr + r] : 0;
    int32_t cnt = 0;
    for (int32_t m = 0; m < n_mol; ++m) cnt += r < n_act ? mnin[(int64_t)m * nc + (int64_t)o * n_pr + ip] : 0;
    double F = r < n_act ? recs[((int64_t)o * n_pr + r) * n_st] : 0.0;
    int32_t partner = -1;
    if (mrg && r < n_act && cnt > 0) {
      const int32_t ipp = mirror[ip];
      const int32_t p = ipp >= 0 ? rmap[ipp] : -1;
      if (p >= 0 && p != r) {
        bool eq = true;
        for (int32_t m = 0; m < n_mol && eq; ++m) {
          const int64_t ca = (int64_t)m * nc + (int64_t)o * n_pr + ip, cb = (int64_t)m * nc + (int64_t)o * n_pr + ipp;
          const int32_t nin = mnin[ca];
          eq = nin == mnin[cb];
          for (int32_t k = 0; k < nin && eq; ++k) {
            const double4 a = msmp[ca * n_x + k], b = msmp[cb * n_x + k];
            eq = __double_as_longlong(a.z) == __double_as_longlong(b.z) && fabs(a.x - b.x) <= kMolMirrorTol &&
                 fabs(a.y - b.y) <= kMolMirrorTol * fmax(fabs(a.y), fabs(b.y));
          }
        }
        if (eq) partner = p;
      }
    }
    // (the lower record of a merged pair carries both weights, the upper one lists nothing)
    if (partner >= 0 && r < partner) F = F + recs[((int64_t)o * n_pr + partner) * n_st];
    const bool skip = partner >= 0 && r > partner;
    const int32_t len = r < n_act ? (skip ? 0 : (fold ? cnt : max(cnt, 1))) : 0;
    const int32_t inc = wave_prefix<int32_t>(len, OpAdd());
    const double fe = wave_prefix<double>(fold && r < n_act && cnt == 0 ? F : 0.0, OpAdd());
    __syncthreads();
    if (lane == 63) { wsum[wid] = inc; wfe[wid] = fe; }
    __syncthreads();
    int32_t pos = base + inc - len, tot = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
      if (w < wid) pos += wsum[w];
      tot += wsum[w];
      fe_sum += wfe[w];
    }
    if (r < n_act && !skip) {
      const int32_t end = pos + len;
      if (cnt == 0 && !fold)
        lo[pos++] = make_double4(0.0, 0.0, __longlong_as_double((long long)(kMolEmpty | kMolLast)), F);
      for (int32_t m = 0; m < n_mol; ++m) {
        const int64_t cidx = (int64_t)m * nc + (int64_t)o * n_pr + ip;
        const int32_t nin = mnin[cidx];
        for (int32_t k = 0; k < nin; ++k) {
          const double4 q = msmp[cidx * n_x + k];
          const bool last = pos == end - 1;
          lo[pos++] = make_double4(q.x, q.y, __longlong_as_double((long long)((last ? kMolLast : 0) | (m << 16) | (int32_t)q.z)),
                                   last ? F : 0.0);
        }
      }
      rend[(int64_t)o * n_pr + r] = end;
    }
    if (r < n_act && skip) rend[(int64_t)o * n_pr + r] = pos;
    base += tot;
  }
  // kMolListPad valid entries past the list (slot 0, P bracket 0, zero weights): k_tau_mol reads its samples in
  // batches without clamping the index
  // (the first one's .w: the folded records' weight sum)
  if (tid < kMolListPad) lo[base + tid] = make_double4(0.0, 0.0, __longlong_as_double(0ll), tid == 0 ? fe_sum : 0.0);
}

void launch_tau_mol(hipStream_t s, TransitDev& tr, RunSlot& rs, int32_t na, dim3, int32_t) {
  // Phase groups: a workgroup runs ppg phases of its 256 wavelengths after a prologue (exp table, first bracket,
  // the LDS stage) worth ~1.4 phases of samples on C5, so fewer, longer groups amortise it, against the tail of the
  // last round of workgroups.  ppg minimises (workgroups / resident slots + 1/2) x (1.4 + ppg) (C5 sweeps,
  // profiles/r05c5b_ppg_sweep.txt: full grid 16 of 32 phases per group, a wavelength shard 8, a 4-phase shard 4;
  // the previous rule, >= 16 waves per SIMD, gave 1, 1 and 8 and a 1.8x slower shard).  PROM_MOL_PPG: fixed.
  const int64_t n_tiles = (tr.n_wav + kBlock - 1) / kBlock;
  // (the CU count of this context's device, cached in its TransitDev: one host thread per device under
  // sumOverChords(devices=...), each with its own context)
  if (tr.cu_count <= 0) {
    int dev = 0, n = 0;
    PROM_HIP(hipGetDevice(&dev));
    PROM_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    tr.cu_count = n > 0 ? n : 256;
  }
  const int cus = tr.cu_count;
  const double slots = 5.0 * cus;   // (k_tau_mol's LDS: five workgroups per CU)
  int32_t ppg = 1;
  double best = 1e300;
  for (int32_t p = 1; p <= tr.n_orb; ++p) {
    const int64_t grp = (tr.n_orb + p - 1) / p;
    if (p > 1 && (tr.n_orb + p - 2) / (p - 1) == grp) continue;   // (same group count: the smaller ppg)
    const double c = ((double)(n_tiles * grp) / slots + 0.5) * (1.4 + (double)p);
    if (c <= best) { best = c; ppg = p; }
  }
  if (const char* e = std::getenv("PROM_MOL_PPG"))
    if (std::atoi(e) > 0) ppg = std::min(tr.n_orb, std::atoi(e));
  const int32_t groups = (tr.n_orb + ppg - 1) / ppg;
  const dim3 g((unsigned)n_tiles, (unsigned)groups);
  const double* wav = tr.wav.as<double>();
  const double* recs = rs.recs.as<double>();
  const int32_t* aip = rs.act_ip.as<int32_t>();
  const double* fo = tr.cfout.as<double>();
  const int32_t* counts = rs.counts.as<int32_t>();
  const double* tf = rs.tsum.as<double>();
  const double* fs = rs.fsum.as<double>();
  double* R = rs.R.as<double>();
    PROM_REQUIRE(na <= 4, "transit: at most 4 atomic constituents next to molecular ones");
    PROM_REQUIRE(tr.n_mol <= 4, "transit: at most 4 molecular constituents");
    for (const auto& md : tr.mslots)
      PROM_REQUIRE(md.n_p < (1 << 15) && (double)std::max(md.n_p - 1, 1) * (double)(md.n_w - 1) * 32.0 < 2147483648.0,
                   "transit: molecular table too large (n_p < 2^15, (n_p - 1) (n_w - 1) 32 bytes < 2^31)");
    // prom_transit_kernel_ms: the kernel's own dispatch-packet events
    hipEvent_t kps = nullptr, kpe = nullptr;
    if (tr.kprof) {
      tr.kprof_mask |= 1u << PROM_K_TAU;
      kps = tr.kprof[2 * PROM_K_TAU];
      kpe = tr.kprof[2 * PROM_K_TAU + 1];
    }
    const int64_t lst_stride = (int64_t)tr.n_pr * (tr.n_mol * tr.n_x + 1) + kMolListPad;
    hipLaunchKernelGGL(k_mol_list, dim3((unsigned)tr.n_orb), dim3(kBlock), 0, s, tr.molslot.as<MolSlotDev>(), tr.n_mol,
                       counts, aip, rs.mol_smp.as<double4>(), rs.mol_nin.as<int32_t>(), recs, 1 + na, tr.n_pr,
                       tr.n_orb, tr.n_x, lst_stride, (int32_t)(na == 0 && tr.exp_mode),
                       tr.n_mirror > 0 && tr.n_pr <= kMolMirrorMax ? tr.mirror.as<int32_t>() : nullptr,
                       rs.mol_lst.as<double4>(), rs.mol_rend.as<int32_t>());
    PROM_HIP(hipGetLastError());
#define PROM_TAUM(NSV, EK)                                                                                  \
  if (tr.n_mol == 1) PROM_TAUM1(NSV, EK, true); else PROM_TAUM1(NSV, EK, false)
#define PROM_TAUM1(NSV, EK, M1V)                                                                            \
  hipExtLaunchKernelGGL((k_tau_mol<NSV, EK, M1V>), g, dim3(kBlock), 0, s, kps, kpe, 0, tr.sigtab_v, tr.molslot.as<MolSlotDev>(), \
                     tr.n_mol, lst_stride, wav, recs, aip, fo, counts, tf, fs, tr.n_pr, tr.n_orb, ppg, tr.n_wav,     \
                     tr.delta_x, rs.mol_lst.as<double4>(), rs.mol_rend.as<int32_t>(), R,                     \
                     tr.count_evals ? rs.evals.as<unsigned long long>() : nullptr, tr.mol_stage ? 1 : 0)
#define PROM_TAUM_NS(EK)                \
  switch (na) {                         \
    case 0: PROM_TAUM(0, EK); break;    \
    case 1: PROM_TAUM(1, EK); break;    \
    case 2: PROM_TAUM(2, EK); break;    \
    case 3: PROM_TAUM(3, EK); break;    \
    default: PROM_TAUM(4, EK);          \
  }
    if (tr.exp_mode) { PROM_TAUM_NS(1) } else { PROM_TAUM_NS(0) }
#undef PROM_TAUM_NS
#undef PROM_TAUM
#undef PROM_TAUM1
}

}  // namespace prom
