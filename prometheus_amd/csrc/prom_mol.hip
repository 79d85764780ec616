// Molecular fused tau kernel (gasProperties.py:924-954 with MolecularConstituent.getSigmaAbs :789-818).
#include "prom_device.h"

namespace prom {

// ---- molecular fused kernel -------------------------------------------------------------------
// tau(c, w) = sum_atomic N_s sigma_s(w) + sum_mol dx * sum_x n_abs(c,x) sigma_m(P(c,x), T, lambda'_w)
// (gasProperties.py:924-954).  Per thread (phase o, wavelength w) and molecular slot, the (T, lambda)
// part of the trilinear RegularGridInterpolator weights is fixed: u_i = sum_{T,lambda corners} w V[i][.][.]
// is formed once for every P node i into LDS; each (chord, sample) then costs one P interpolation
// (uniform bracket from k_mol_prep), 10^v and an FMA.  Out-of-table samples (P, T or lambda) take the
// fill value, i.e. sigma = 0, as in the reference.
constexpr double kLog2Ten256 = 0x1.a934f0979a371p+9;    // 256 log2(10)
constexpr int kMolExpN = 256;                              // LDS exp table 2^(i/256) (2 KB: occupancy)

// 2^(y/256) = 2^(k >> 8) T[k & 255] exp(d ln2/256), k = rint(y), d in [-1/2, 1/2], degree-5 Taylor
// polynomial (truncation 9e-21 relative; acc_exp256's arithmetic without the accumulation)
__device__ __forceinline__ double exp2_256(double y, const double* __restrict__ tab) {
  const double k = __builtin_rint(y);
  const int ki = (int)k;
  const double d = y - k;
  double p = __builtin_fma(d, kE256C5, kE256C4);
  p = __builtin_fma(d, p, kE256C3);
  p = __builtin_fma(d, p, kE256C2);
  p = __builtin_fma(d, p, kE256C1);
  p = __builtin_fma(d, p, 1.0);
  return __builtin_amdgcn_ldexp(tab[ki & (kMolExpN - 1)], ki >> 8) * p;
}

template <int NSA, int EXPK>
__global__ void __launch_bounds__(kBlock) k_tau_mol(const SigTabs4 tabv, const SigTabDev* __restrict__ tabs,
                                                    const MolSlotDev* __restrict__ ms, int32_t n_mol,
                                                    int32_t max_np, int64_t lst_stride,
                                                    const double* __restrict__ wav,
                                                    const double* __restrict__ recs,
                                                    const int32_t* __restrict__ act_ip,
                                                    const double* __restrict__ fout,
                                                    const int32_t* __restrict__ counts,
                                                    const double* __restrict__ tfrac,
                                                    const double* __restrict__ fsum, int32_t n_pr,
                                                    int32_t n_orb, int32_t phases_per_group, int64_t n_wav,
                                                    int32_t n_x, double delta_x,
                                                    const double4* __restrict__ lst,
                                                    const int32_t* __restrict__ rend, double* __restrict__ R,
                                                    unsigned long long* __restrict__ evals) {
  extern __shared__ double lds[];   // [256] exp table 2^(i/256) | [n_mol][max_np][kBlock] u
  double* etab = lds;
  double* ul = lds + kMolExpN;
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
  int64_t whint[4] = {-1, -1, -1, -1};
  unsigned long long npow = 0;   // stats runs: this lane's 10^v evaluations (in-table samples)

  uint32_t inb = 0;              // bit m: molecular slot m has (T, lambda') inside its table
  double lwprev[4];              // slot m's lambda' of the last u built in LDS (m < 4)
#pragma unroll
  for (int m = 0; m < 4; ++m) lwprev[m] = __builtin_nan("");
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
    for (int32_t m = 0; m < n_mol; ++m) {
      const MolSlotDev d = ms[m];
      int64_t it, iw;
      double tt, tw;
      const double lw = d.shift[o] * lam;
      // the same lambda' as this lane's previous phase (no orbital Doppler shift, or an equal factor): u and
      // the in-table bit are unchanged (T is the slot's own constant)
      if (m < 4) {
        if (lw == lwprev[m]) continue;
        lwprev[m] = lw;
      }
      inb &= ~(1u << m);
      bool ok = rgi_bracket(d.T, d.n_t, d.temp, &it, &tt);
      if (ok) {
        // gallop the wavelength bracket from the previous phase's
        ok = lw >= d.W[0] && lw <= d.W[d.n_w - 1];
        if (ok) {
          int64_t h = m < 4 ? whint[m] : -1;
          int64_t lo = 0, hi = d.n_w - 1;
          if (h >= 0 && h <= d.n_w - 2 && d.W[h] < lw && lw <= d.W[h + 1]) { lo = h; hi = h + 1; }
          // scipy: i = searchsorted(g, v, 'left') - 1 clipped to [0, n-2]
          while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if (d.W[mid] < lw) lo = mid; else hi = mid;
          }
          iw = lo;
          if (lw <= d.W[0]) iw = 0;
          tw = (lw - d.W[iw]) / (d.W[iw + 1] - d.W[iw]);
          if (m < 4) whint[m] = iw;
        }
      }
      if (ok) {
        inb |= 1u << m;
        const double w00 = (1.0 - tt) * (1.0 - tw), w01 = (1.0 - tt) * tw;
        const double w10 = tt * (1.0 - tw), w11 = tt * tw;
        for (int32_t i = 0; i < d.n_p; ++i) {
          const double* v0 = d.V + ((int64_t)i * d.n_t + it) * d.n_w + iw;
          const double* v1 = v0 + d.n_w;
          double u = 0.0;
          u = u + v0[0] * w00;
          u = u + v0[1] * w01;
          u = u + v1[0] * w10;
          u = u + v1[1] * w11;
          ul[((int64_t)m * max_np + i) * kBlock + threadIdx.x] = u;
        }
      }
    }
    const int32_t* ipl = act_ip + (int64_t)o * n_pr;
    double acc = 0.0;
    const double scale = exact ? 1.0 : kM256Ln2;
    // The phase's in-table samples are one flat list in record order (k_mol_list: {P weight, n_abs, slot << 16 |
    // P bracket, offset}, record r's samples ending at rend[r]), read with wave-uniform scalar loads four at a
    // time: the four samples' u reads, 10^v and products are independent; then they are added into the current
    // record's sum, finishing records (e^-tau) at their ends.  Per sample n_abs (10^v - offset), the reference's
    // order of the subtraction (gasProperties.py:811-818, 10**interp - offset).
    const double4* __restrict__ lo = lst + (int64_t)o * lst_stride;
    const int32_t* __restrict__ ro = rend + (int64_t)o * n_pr;
    const int32_t K = n_act > 0 ? ro[n_act - 1] : 0;
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
      if (!exact) acc = acc_exp256(acc, rr[0], tau * scale, etab);
      else acc = acc + fout[ipl[ri]] * exp(-tau);
    };
    for (int32_t k0 = 0; k0 < K; k0 += 4) {
      double c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int32_t k = k0 + j < K ? k0 + j : K - 1;
        const double4 q = lo[k];
        const int32_t code = (int32_t)q.z;
        const int32_t m = code >> 16, pi = code & 0xffff;
        const double* um = ul + ((int64_t)m * max_np + pi) * kBlock + threadIdx.x;
        const double a = um[0], b = um[kBlock];
        double e;
        if (EXPK && !exact) {
          // 10^v = 2^(y/256), y = v 256 log2(10), from the LDS table (relative error ~ |y| 2^-53 ln2/256 from the
          // argument, ~1e-14 at the table's floor)
          e = exp2_256(__builtin_fma(q.x, b - a, a) * kLog2Ten256, etab);
        } else {
          e = exp10((1.0 - q.x) * a + q.x * b);
        }
        const bool in = ((inb >> m) & 1u) != 0;
        c[j] = in ? q.y * (e - q.w) : 0.0;
        npow += (in && k0 + j < K) ? 1u : 0u;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
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
          lo[pos++] = make_double4(q.x, q.y, (double)((m << 16) | (int32_t)q.z), off);
        }
      }
      rend[(int64_t)o * n_pr + r] = pos;
    }
    base += tot;
  }
}

void launch_tau_mol(hipStream_t s, TransitDev& tr, RunSlot& rs, int32_t na, dim3 g, int32_t ppg) {
  const SigTabDev* tabs = tr.sigtab.as<SigTabDev>();
  const double* wav = tr.wav.as<double>();
  const double* recs = rs.recs.as<double>();
  const int32_t* aip = rs.act_ip.as<int32_t>();
  const double* fo = tr.cfout.as<double>();
  const int32_t* counts = rs.counts.as<int32_t>();
  const double* tf = rs.tsum.as<double>();
  const double* fs = rs.fsum.as<double>();
  double* R = rs.R.as<double>();
    PROM_REQUIRE(na <= 4, "transit: at most 4 atomic constituents next to molecular ones");
    int32_t max_np = 0;
    for (const auto& m : tr.mslots) max_np = std::max(max_np, m.n_p);
    const size_t lds = kMolExpN * sizeof(double) + (size_t)tr.n_mol * max_np * kBlock * sizeof(double);
    PROM_REQUIRE(lds <= 160 * 1024, "transit: molecular tables too large for the LDS staging (n_mol * n_p)");
    PROM_REQUIRE(tr.n_mol <= 4, "transit: at most 4 molecular constituents");
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
  hipExtLaunchKernelGGL((k_tau_mol<NSV, EK>), g, dim3(kBlock), lds, s, kps, kpe, 0, tr.sigtab_v, tabs, tr.molslot.as<MolSlotDev>(), tr.n_mol, \
                     max_np, lst_stride, wav, recs, aip, fo, counts, tf, fs, tr.n_pr, tr.n_orb, ppg, tr.n_wav, tr.n_x, \
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
}

}  // namespace prom
