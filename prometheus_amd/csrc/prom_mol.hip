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

// 2^(y/1024) = 2^(k >> 10) T[k & 1023] exp(d ln2/1024), k = rint(y), d in [-1/2, 1/2], cubic Taylor polynomial
// (truncation 5.5e-16 relative; acc_exp1024's arithmetic without the accumulation)
__device__ __forceinline__ double exp2_1024(double y, const double* __restrict__ tab) {
  const double k = __builtin_rint(y);
  const int ki = (int)k;
  const double d = y - k;
  double p = __builtin_fma(d, kE1024C3, kE1024C2);
  p = __builtin_fma(d, p, kE1024C1);
  p = __builtin_fma(d, p, 1.0);
  return __builtin_amdgcn_ldexp(tab[ki & (kMolExpN - 1)], ki >> 10) * p;
}

// G of one slot: [n_p][n_w - 1] pairs {g(i, w), g(i, w + 1)} at the slot's T (unused when T is outside the table)
__global__ void k_mol_gt(const double* __restrict__ Tg, int32_t n_t, double T, const double* __restrict__ V,
                         int32_t n_p, int64_t n_w, double2* __restrict__ G) {
  int64_t it = 0;
  double tt = 0.0;
  if (!rgi_bracket(Tg, n_t, T, &it, &tt)) return;
  const int64_t nw1 = n_w - 1;
  const int64_t tot = (int64_t)n_p * nw1;
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < tot; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = k / nw1, w = k - i * nw1;
    const double* v0 = V + (i * n_t + it) * n_w + w;
    const double* v1 = v0 + n_w;
    // stored as y = 1024 log2(10) v (the lookups' exponent scale: 10^v = 2^(y/1024), no multiply per sample)
    G[k] = make_double2(((1.0 - tt) * v0[0] + tt * v1[0]) * kLog2Ten1024, ((1.0 - tt) * v0[1] + tt * v1[1]) * kLog2Ten1024);
  }
}

void launch_mol_gt(hipStream_t s, const MolSlotDev& md) {
  const int64_t tot = (int64_t)md.n_p * (md.n_w - 1);
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
                                                    unsigned long long* __restrict__ evals) {
  __shared__ double etab[kMolExpN];   // exp table 2^(i/1024)
  if (EXPK)
    for (int i = threadIdx.x; i < kMolExpN; i += kBlock) etab[i] = kExp2TableDev[i * (PROM_EXP2_TABLE_N / kMolExpN)];
  __syncthreads();
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
#pragma unroll
  for (int m = 0; m < (M1 ? 1 : 4); ++m) {
    const bool valid = m < n_mol;   // (unused slots: empty buffers, never selected)
    int64_t it;
    double tt;
    if (valid && rgi_bracket(ms[m].T, ms[m].n_t, ms[m].temp, &it, &tt)) tin |= 1u << m;
    rowbv[m] = valid ? (uint32_t)(ms[m].n_w - 1) * (uint32_t)sizeof(double2) : 0u;
    rsv[m] = __builtin_amdgcn_make_buffer_rsrc(valid ? const_cast<double2*>(ms[m].G) : nullptr, (short)0,
                                               valid ? (int)((uint32_t)ms[m].n_p * rowbv[m]) : 0, 0x00020000);
  }
  int64_t iwv[4] = {-1, -1, -1, -1};
  double twv[4] = {0.0, 0.0, 0.0, 0.0};
  uint32_t inb = 0;
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
      const double lw = ms[m].shift[o] * lam;
      // scipy: i = searchsorted(W, lw, 'left') - 1 clipped to [0, n-2], fill outside [W[0], W[n-1]]
      const bool ok = ((tin >> m) & 1u) && lw >= W[0] && lw <= W[nw - 1];
      inb = ok ? (inb | (1u << m)) : (inb & ~(1u << m));
      if (!ok) continue;
      int64_t h = iwv[m];
      if (h < 0) {
        int64_t lo = 0, hi = nw - 1;
        while (hi - lo > 1) {
          const int64_t mid = (lo + hi) >> 1;
          if (W[mid] < lw) lo = mid; else hi = mid;
        }
        h = lo;
      } else {
        // walk from the previous phase's bracket (adjacent phases' Doppler factors differ by ~1e-6)
        while (h < nw - 2 && W[h + 1] < lw) ++h;
        while (h > 0 && !(W[h] < lw)) --h;
      }
      iwv[m] = h;
      twv[m] = (lw - W[h]) / (W[h + 1] - W[h]);
    }
    const int32_t* ipl = act_ip + (int64_t)o * n_pr;
    double acc = 0.0;
    // The phase's in-table samples are one flat list in record order (k_mol_list: {P weight, n_abs, slot << 16 |
    // P bracket, offset}, record r's samples ending at rend[r]), read with wave-uniform scalar loads four at a
    // time: the four samples' G reads, 10^v and products are independent; then they are added into the current
    // record's sum, finishing records (e^-tau) at their ends.  Per sample n_abs (10^v - offset), the reference's
    // order of the subtraction (gasProperties.py:811-818, 10**interp - offset).
    const double4* __restrict__ lo = lst + (int64_t)o * lst_stride;
    const int32_t* __restrict__ ro = rend + (int64_t)o * n_pr;
    const int32_t K = n_act > 0 ? ro[n_act - 1] : 0;
    // per slot: the lane's byte offset of its lambda' pair in a G row and the in-table mask (1 / 0: a product, no
    // select; out-of-table lanes read the row's first pair, finite)
    uint32_t boff[M1 ? 1 : 4];
    double msk[M1 ? 1 : 4];
#pragma unroll
    for (int m = 0; m < (M1 ? 1 : 4); ++m) {
      const bool in = ((inb >> m) & 1u) != 0;
      boff[m] = in ? (uint32_t)iwv[m] * (uint32_t)sizeof(double2) : 0u;
      msk[m] = in ? 1.0 : 0.0;
    }
    int32_t nsl[4] = {0, 0, 0, 0};   // samples per slot (uniform; stats)
    // one instance per exp mode (uniform per phase), so the four samples' loads issue together
    auto samples = [&](auto ex) {
      constexpr bool EX = decltype(ex)::value;
      int32_t r = 0;
      int32_t end_r = n_act > 0 ? ro[0] : 0;
      double sm = 0.0;
      auto finish = [&](int32_t ri) {
        const double* rr = rec + (int64_t)ri * ST;
        double tau = 0.0;
#pragma unroll
        for (int s = 0; s < NSA; ++s) tau = tau + rr[1 + s] * sg[s];
        tau = tau + sm * delta_x;
        sm = 0.0;
        if constexpr (!EX) acc = acc_exp1024(acc, rr[0], tau * kM1024Ln2, etab);
        else acc = acc + fout[ipl[ri]] * exp(-tau);
      };
      constexpr int NB = EX ? 1 : 4;   // (the ocml exp10 path: one sample at a time, few registers)
      for (int32_t k0 = 0; k0 < K; k0 += NB) {
        double c[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const int32_t k = k0 + j < K ? k0 + j : K - 1;
          const double4 q = lo[k];
          const int32_t code = (int32_t)__double_as_longlong(q.z);   // (integer bits: scalar decode)
          const int32_t m = M1 ? 0 : code >> 16, pi = code & 0xffff;
          // the slot's bracket (m uniform: selects, no indexing of the register arrays)
          uint32_t bo = boff[0];
          double tw = twv[0], mk = msk[0];
          __amdgpu_buffer_rsrc_t rs = rsv[0];
          uint32_t rowb = rowbv[0];
          if constexpr (!M1) {
#pragma unroll
            for (int mm = 1; mm < 4; ++mm)
              if (m == mm) { bo = boff[mm]; tw = twv[mm]; mk = msk[mm]; rs = rsv[mm]; rowb = rowbv[mm]; }
            if (k0 + j < K) nsl[m & 3] += 1;
          }
          // rows pi and pi + 1: buffer loads, the row at a uniform offset (soffset), the lane's pair at its own
          const uint32_t so = (uint32_t)pi * rowb;
          const double2 ga = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, bo, so, 0));
          const double2 gb = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rs, bo, so + rowb, 0));
          const double a = __builtin_fma(tw, ga.y - ga.x, ga.x);
          const double b = __builtin_fma(tw, gb.y - gb.x, gb.x);
          const double v = __builtin_fma(q.x, b - a, a);
          double e;
          if constexpr (!EX) {
            // 10^v = 2^(y/1024), y = v 1024 log2(10), from the LDS table (relative error ~ |v| ln10 2^-53 from the
            // argument, ~6e-15 at the table's floor)
            e = exp2_1024(v, etab);
          } else {
            // (v is 1024 log2(10) times the table value: 2^(v/1024) = 10^value.  The scaling of G, k_mol_gt, adds
            // |value| ln10 2^-53 relative per sample (8e-15 at -30) next to ocml's exp2; the validation test
            // test_transit_ocml_exp_mode checks this path against the reference's golden R at 1e-12)
            e = exp2(v * 0x1p-10);
          }
          c[j] = (q.y * (e - q.w)) * mk;
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const int32_t k = k0 + j;
          if (k >= K) break;
          while (k >= end_r) {
            finish(r);
            ++r;
            end_r = ro[r];
          }
          sm += c[j];
        }
      }
      for (; r < n_act; ++r) finish(r);
    };
    if (!EXPK || exact) samples(std::true_type{});
    else samples(std::false_type{});
    if (evals) {
      if constexpr (M1) nsl[0] = K;
#pragma unroll
      for (int m = 0; m < 4; ++m) npow += ((inb >> m) & 1u) ? (unsigned long long)nsl[m] : 0ull;
    }
    if (live) R[(int64_t)o * n_wav + w] = exact ? (acc + tfrac[o] * fsum[o]) / fsum[o] : acc + tfrac[o];
  }
  if (evals && live && npow) atomicAdd(&evals[(blockIdx.x * 4 + (threadIdx.x >> 6)) & 63], npow);
}

// Per phase: the in-table samples of its records (k_chords' active chords, chord order) as one flat list for
// k_tau_mol: record r's samples of every molecular slot (k_mol_prep's compacted rows) at [rend[r - 1], rend[r]),
// each {P weight, n_abs, slot << 16 | P bracket, the slot's offset}.  One workgroup per phase.
__global__ void __launch_bounds__(kBlock) k_mol_list(const MolSlotDev* __restrict__ ms, int32_t n_mol,
                                                     const int32_t* __restrict__ counts,
                                                     const int32_t* __restrict__ act_ip,
                                                     const double4* __restrict__ msmp,
                                                     const int32_t* __restrict__ mnin, int32_t n_pr, int32_t n_orb,
                                                     int32_t n_x, int64_t lst_stride, double4* __restrict__ lst,
                                                     int32_t* __restrict__ rend) {
  __shared__ int32_t wsum[kBlock / 64];
  const int32_t o = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int32_t n_act = counts[o * kCnt];
  const int64_t nc = (int64_t)n_orb * n_pr;
  double4* lo = lst + (int64_t)o * lst_stride;
  int32_t base = 0;
  for (int32_t r0 = 0; r0 < n_act; r0 += kBlock) {
    const int32_t r = r0 + tid;
    const int32_t ip = r < n_act ? act_ip[(int64_t)o * n_pr + r] : 0;
    int32_t cnt = 0;
    for (int32_t m = 0; m < n_mol; ++m) cnt += r < n_act ? mnin[(int64_t)m * nc + (int64_t)o * n_pr + ip] : 0;
    const int32_t inc = wave_prefix<int32_t>(cnt, OpAdd());
    __syncthreads();
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    int32_t pos = base + inc - cnt, tot = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
      if (w < wid) pos += wsum[w];
      tot += wsum[w];
    }
    if (r < n_act) {
      for (int32_t m = 0; m < n_mol; ++m) {
        const int64_t cidx = (int64_t)m * nc + (int64_t)o * n_pr + ip;
        const int32_t nin = mnin[cidx];
        const double off = ms[m].offset;
        for (int32_t k = 0; k < nin; ++k) {
          const double4 q = msmp[cidx * n_x + k];
          lo[pos++] = make_double4(q.x, q.y, __longlong_as_double((long long)((m << 16) | (int32_t)q.z)), off);
        }
      }
      rend[(int64_t)o * n_pr + r] = pos;
    }
    base += tot;
  }
}

void launch_tau_mol(hipStream_t s, TransitDev& tr, RunSlot& rs, int32_t na, dim3, int32_t) {
  // phase groups: at least ~16 waves per SIMD over the whole grid (65,536 over 1,024 SIMDs), so the last round of
  // the equally long waves is a small tail (one group of all 32 C5 phases left a 4th round ~5 % full: 1.58x on
  // the step against 4-phase pieces, BENCH_r03 phase_shard); each group's first phase binary-searches the lambda'
  // bracket, the others walk it.  PROM_MOL_PPG (profiling): phases per group.
  const int64_t n_tiles = (tr.n_wav + kBlock - 1) / kBlock;
  int32_t groups = (int32_t)std::max<int64_t>(1, std::min<int64_t>(tr.n_orb, (65536 + 4 * n_tiles - 1) / (4 * n_tiles)));
  int32_t ppg = (tr.n_orb + groups - 1) / groups;
  // equal groups: the next phase count that divides the phases (C5: 7 -> 8, four groups of 8; a short last group
  // ends early and leaves its CUs idle: profiles/r04o_C5_ppg_sweep.txt)
  while (ppg < tr.n_orb && tr.n_orb % ppg != 0 && ppg < 2 * ((tr.n_orb + groups - 1) / groups)) ++ppg;
  if (const char* e = std::getenv("PROM_MOL_PPG"))
    if (std::atoi(e) > 0) ppg = std::min(tr.n_orb, std::atoi(e));
  groups = (tr.n_orb + ppg - 1) / ppg;
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
      PROM_REQUIRE(md.n_p < (1 << 15) && (double)md.n_p * (double)(md.n_w - 1) * 16.0 < 2147483648.0,
                   "transit: molecular table too large (n_p < 2^15, n_p (n_w - 1) 16 bytes < 2^31)");
    // prom_transit_kernel_ms: the kernel's own dispatch-packet events
    hipEvent_t kps = nullptr, kpe = nullptr;
    if (tr.kprof) {
      tr.kprof_mask |= 1u << PROM_K_TAU;
      kps = tr.kprof[2 * PROM_K_TAU];
      kpe = tr.kprof[2 * PROM_K_TAU + 1];
    }
    const int64_t lst_stride = (int64_t)tr.n_pr * tr.n_mol * tr.n_x;
    hipLaunchKernelGGL(k_mol_list, dim3((unsigned)tr.n_orb), dim3(kBlock), 0, s, tr.molslot.as<MolSlotDev>(), tr.n_mol,
                       counts, aip, tr.mol_smp.as<double4>(), tr.mol_nin.as<int32_t>(), tr.n_pr, tr.n_orb, tr.n_x,
                       lst_stride, tr.mol_lst.as<double4>(), tr.mol_rend.as<int32_t>());
    PROM_HIP(hipGetLastError());
#define PROM_TAUM(NSV, EK)                                                                                  \
  if (tr.n_mol == 1) PROM_TAUM1(NSV, EK, true); else PROM_TAUM1(NSV, EK, false)
#define PROM_TAUM1(NSV, EK, M1V)                                                                            \
  hipExtLaunchKernelGGL((k_tau_mol<NSV, EK, M1V>), g, dim3(kBlock), 0, s, kps, kpe, 0, tr.sigtab_v, tr.molslot.as<MolSlotDev>(), \
                     tr.n_mol, lst_stride, wav, recs, aip, fo, counts, tf, fs, tr.n_pr, tr.n_orb, ppg, tr.n_wav,     \
                     tr.delta_x, tr.mol_lst.as<double4>(), tr.mol_rend.as<int32_t>(), R,                     \
                     tr.count_evals ? rs.evals.as<unsigned long long>() : nullptr)
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
