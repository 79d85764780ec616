// The transmission-curve path: the default for one effective absorber (merged species or one species).
//
// With one absorber every chord's optical depth is tau_c(o, w) = N_c Y(o, w): its column N_c times the
// absorber's cross-section Y(o, w) = sum_s chi_s sigma_s(shift_o lambda_w) (gasProperties.py:941-954, the
// reference's tau += N_s sigma_s).  The disk sum of sumOverChords (gasProperties.py:1241-1258) is then one
// function of one variable per phase:
//
//   R(o, w) = T_o(Y(o, w)),   T_o(Y) = tfrac_o + sum_{active c} F_c exp(-N_c Y),   F_c = F_out,c / sum F_out,
//
// the phase's transmission curve.  Per run:
//   k_columns8   columns and culling (prom_transit.hip);
//   k_tc_build   per (phase, chain of 4 octaves of q = Y N_max, part of the chords): the phase's sums, tfrac,
//                N_max, the tail polynomial's coefficients, and T_o at 16 Chebyshev nodes of log2 q per octave
//                (exact sums over every active chord) turned into 16 Chebyshev coefficients;
//   k_sigma_tc   per (phase, wavelength): Y from the Doppler-shifted table lookups, then T_o(Y) -> R.
// T_o is evaluated three ways:
//   q < 2^-7      every chord has tau = n_c q <= q (n_c = N_c / N_max <= 1): degree-5 Taylor polynomial of
//                 exp(-tau) summed over the chords, t_e = (-1)^e sum_c F_c n_c^e / e!; truncation <= q^6/720
//                 <= 3.2e-16 per unit weight (C3: 99 % of the points);
//   octave j      q in [2^(j-7), 2^(j-6)): degree-15 Chebyshev series in v = log2(q) - (j - 7); the
//                 interpolation error of g(s) = exp(-e^s) on one octave of s = ln q + ln n_c is below
//                 2 max|g^(16)| (ln2/2)^16 / (2^15 16!) = 3e-17 per unit weight for any set of columns;
//   above         q >= 40 N_max / N_min: every tau >= 40, T_o = tfrac within e^-40; otherwise (a table
//                 truncated at the host's octave cap) the exact sum over the phase's chords.
// So |R - R_exact| is a few 1e-16 plus the rounding of the sums, against the windowed path's 4e-14.  A phase
// with a non-finite column takes the reference's chord order with ocml exp (the NaN pattern), as before.
//
// Codegen dependence (k_tc_build's hand-off between the parts of a (phase, chain)): the parts' sums are published
// with relaxed agent-scope atomic stores, which gfx950 emits as write-through global_store ... sc1, each storing wave
// waits vmcnt(0), then one agent-scope atomic add per workgroup; the last arriver reads with relaxed agent-scope
// atomic loads (global_load ... sc1).  This is MI355X_MICROARCH.md's measured sc1 form, used in place of an
// agent-scope release/acquire pair (whose release is a buffer_wbl2 of the whole XCD L2: 1.7-6.5 us per workgroup and
// run).  It relies on the relaxed agent-scope atomics compiling to sc1 accesses; a compiler that lowered them
// otherwise would need the fences back.  tests/test_gpu_tcurve.py (curves against the exact sums, many parts) would
// show a stale partial sum as a wrong curve.
#include "prom_tc.h"

namespace prom {

// Reductions over the 64 lanes of a wavefront on DPP moves (quad permutes, half-row and row mirrors) and four
// readlanes: no LDS round trips, a fixed combination order, a wave-uniform result.
template <typename T, typename Op>
__device__ __forceinline__ T tc_wred(T v, Op op) {
  v = op(v, dpp_mov<0xB1>(v));    // quad_perm [1,0,3,2]
  v = op(v, dpp_mov<0x4E>(v));    // quad_perm [2,3,0,1]
  v = op(v, dpp_mov<0x141>(v));   // row_half_mirror
  v = op(v, dpp_mov<0x140>(v));   // row_mirror: every lane of a row holds the row's fold
  return op(op(lane_read(v, 0), lane_read(v, 16)), op(lane_read(v, 32), lane_read(v, 48)));
}
struct OpAddI { __device__ int32_t operator()(int32_t a, int32_t b) const { return a + b; } };

// ---- per phase: sums, tail coefficients and the transmission-curve table, in one kernel ------------------
// Grid (chain, part, phase).  Every workgroup first takes the phase's sums over all its chords (F_out sum,
// transparent sum, N_max / N_min over the active finite columns, counts; one strided sweep, L2-resident
// inputs) and the table extent L, identically.  Then part p of the chords [c_p, c_{p+1}) and chain ch of
// octaves 4 ch .. 4 ch + 3: thread (k, g) = (t & 15, t >> 4) evaluates e = exp(-N q_k / N_max) at node k of
// octave 4 ch for chords c_p + g, c_p + g + 16, ... and the next three octaves by squaring (q doubles from one
// octave to the next: e^{-2x} = (e^{-x})^2; three squarings carry <= 2^3 (3u) + 7u = 31u = 3.4e-15 relative
// error), so one table exp serves four octaves.  Chain 0 also sums the tail moments sum F n^e.  The parts'
// node sums go to `part`; the last part to finish (atomic counter per (phase, chain), reset by it) adds them in
// part order -- deterministic -- and writes the Chebyshev coefficients (and, chain 0, the header).
constexpr int kTcB2 = 256;               // threads per workgroup (16 groups of 16 node threads)
constexpr int kTcPartLds = 1024;         // a part's chords staged in LDS up to this many (16 KB)
#ifndef PROM_TC_ILP
#define PROM_TC_ILP 4                    // node sums: chords per iteration (build macro, for sweeps)
#endif
static_assert(kTcPartVals == (kTcChain + 1) * kTcD, "per part: 4 octaves' node sums, then the moments' row");

__device__ __forceinline__ double exp256(double y, const double* __restrict__ tab) {
  // 2^(y/256) for y = -x 256/ln2 (acc_exp256's arithmetic without the accumulation)
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

__global__ void __launch_bounds__(kTcB2) k_tc_build(const int32_t* __restrict__ flags, const double* __restrict__ fout,
                                                   const double* __restrict__ ncol, int32_t n_pr, int32_t n_parts,
                                                   double ybound, int32_t lg, const double* __restrict__ tcc,
                                                   double* __restrict__ hdr,
                                                   double* __restrict__ tab, double* __restrict__ part,
                                                   int32_t* __restrict__ cnt, int32_t* __restrict__ counts,
                                                   unsigned long long* __restrict__ evals,
                                                   const TcPart* __restrict__ tcp, double fsum_set) {
  constexpr int NW = kTcB2 / 64;
  const int32_t ch = blockIdx.x, pt = blockIdx.y, o = blockIdx.z;
  const int32_t n_ch = gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
#ifdef PROM_TRACE
  // per workgroup (tools/trace_tcb.py), at g_trace[2^19 + 8 id]: wall clock at start, after the phase sums, after
  // the node sums, after the hand-off, at the end; then ch | part << 8 | phase << 16, L | last << 16
  unsigned long long* tq = g_trace + (1u << 19) + 8ull * ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x);
  if (tid == 0) tq[0] = wall_clock64();
  __shared__ unsigned long long s_tmax[2];   // the slowest wave's end of the sweep / of the node sums
  if (tid == 0) s_tmax[0] = s_tmax[1] = 0;
  __syncthreads();
#endif
  __shared__ double etab[256];
  __shared__ double sd[4][NW];
  __shared__ int32_t si[4][NW];
  __shared__ double red[NW][kTcChain + 1][kTcD];
  __shared__ double sf[kTcChain + 1][kTcD];
  __shared__ int32_t s_last;
  __shared__ double2 spart[kTcPartLds];
  const int32_t* fl = flags + (int64_t)o * n_pr;
  const double* nc = ncol + (int64_t)o * n_pr;
  // the exp table (the Chebyshev matrix and the node factors come precomputed: tcc)
  if (tid < 256) etab[tid] = kExp2TableDev[8 * tid];
  // 1. the phase's sums (every workgroup of the phase, the same order).  Sweeps of kTcB2 x U chords, every load
  // of a sweep issued before any is used (one round trip per sweep, no load behind a flag test); this part's
  // chords [c_lo, c_hi) are kept in LDS on the way ({F_out, N}, zero for inactive chords) for step 2
  const int32_t c_lo = (int32_t)((int64_t)n_pr * pt / n_parts), c_hi = (int32_t)((int64_t)n_pr * (pt + 1) / n_parts);
  const bool in_lds = c_hi - c_lo <= kTcPartLds;
  double fs = 0.0, ts = 0.0, nmax = 0.0, nmin = __builtin_inf();
  int32_t nact = 0, ntr = 0, nbl = 0, nnf = 0;
  constexpr int U = 12;   // (one sweep up to 3072 chords)
  if (tcp) {
    // k_columns8's partials (32 chords each: max / min / counts, order-independent) instead of a sweep over every
    // chord; only this part's chords are loaded (to LDS, with their transparent F_out sum: the phase's comes from the
    // parts in part order); the F_out total is the set's
    const int32_t n_g = n_pr / 32;
    for (int32_t g = tid; g < n_g; g += kTcB2) {
      const TcPart v = tcp[(int64_t)o * n_g + g];
      nmax = v.nmax > nmax ? v.nmax : nmax;
      nmin = v.nmin < nmin ? v.nmin : nmin;
      nact += v.nact; ntr += v.ntr; nbl += v.nbl; nnf += v.nnf;
    }
    for (int32_t c = c_lo + tid; c < c_hi; c += kTcB2) {
      const int32_t f = fl[c];
      const double fo = fout[c], N = nc[c];
      if (in_lds) spart[c - c_lo] = f == 0 ? make_double2(fo, N) : make_double2(0.0, 0.0);
      ts += f == 1 ? fo : 0.0;
    }
  }
  for (int32_t c0 = 0; !tcp && c0 < n_pr; c0 += kTcB2 * U) {
    int32_t f[U];
    double fo[U], N[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int32_t c = min(c0 + u * kTcB2 + tid, n_pr - 1);   // (clamped: no branch around the loads)
      f[u] = fl[c];
      fo[u] = fout[c];
      N[u] = nc[c];
    }
    // branch-free accumulation (selects; a chord past n_pr adds nothing)
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int32_t c = c0 + u * kTcB2 + tid;
      const bool valid = c < n_pr;
      const bool act = valid && f[u] == 0, tra = valid && f[u] == 1;
      const bool fin_n = __builtin_isfinite(N[u]);
      fs += valid ? fo[u] : 0.0;
      ts += tra ? fo[u] : 0.0;
      ntr += tra ? 1 : 0;
      nbl += (valid && f[u] == 2) ? 1 : 0;
      nact += act ? 1 : 0;
      nnf += (act && !fin_n) ? 1 : 0;
      nmax = (act && fin_n && N[u] > nmax) ? N[u] : nmax;
      nmin = (act && fin_n && N[u] > 0.0 && N[u] < nmin) ? N[u] : nmin;
      if (in_lds && c >= c_lo && c < c_hi) spart[c - c_lo] = act ? make_double2(fo[u], N[u]) : make_double2(0.0, 0.0);
    }
  }
#ifdef PROM_TRACE
  if (lane == 0) {   // (the slowest wave, after its sweep's loads are used)
    double x = fs;
    asm volatile("" : "+v"(x));
    atomicMax(&s_tmax[0], wall_clock64());
  }
#endif
  fs = tc_wred<double>(fs, OpAdd());
  ts = tc_wred<double>(ts, OpAdd());
  nmax = tc_wred<double>(nmax, OpMax());
  nmin = tc_wred<double>(nmin, OpMin());
  nact = tc_wred<int32_t>(nact, OpAddI());
  ntr = tc_wred<int32_t>(ntr, OpAddI());
  nbl = tc_wred<int32_t>(nbl, OpAddI());
  nnf = tc_wred<int32_t>(nnf, OpAddI());
  if (lane == 0) {
    sd[0][wid] = fs; sd[1][wid] = ts; sd[2][wid] = nmax; sd[3][wid] = nmin;
    si[0][wid] = nact; si[1][wid] = ntr; si[2][wid] = nbl; si[3][wid] = nnf;
  }
  __syncthreads();
  fs = sd[0][0]; ts = sd[1][0]; nmax = sd[2][0]; nmin = sd[3][0];   // (tcp: ts is this part's)
  nact = si[0][0]; ntr = si[1][0]; nbl = si[2][0]; nnf = si[3][0];
#pragma unroll
  for (int w = 1; w < NW; ++w) {
    fs += sd[0][w]; ts += sd[1][w];
    nmax = sd[2][w] > nmax ? sd[2][w] : nmax;
    nmin = sd[3][w] < nmin ? sd[3][w] : nmin;
    nact += si[0][w]; ntr += si[1][w]; nbl += si[2][w]; nnf += si[3][w];
  }
  if (tcp) fs = fsum_set;
  // table extent: octaves up to the host's bound of q = Y N_max, or up to q = 40 N_max / N_min (every chord
  // opaque beyond it), whichever comes first; lg caps it
  const bool fin = nnf == 0 && nmax > 0.0 && nact > 0;
  int32_t L = 0, top_opaque = 0, trunc = 0;
  if (fin) {
    const int32_t L1 = ybound > 0.0 ? tc_octaves(ybound * nmax * (1.0 + 0x1p-40)) : 0x7fffffff;
    const int32_t L2 = tc_octaves(kTcSat * (nmax / nmin));
    if (L2 <= L1 && L2 <= lg) {
      L = L2;
      top_opaque = 1;
    } else {
      L = L1 < lg ? L1 : lg;
      trunc = L1 > lg ? 4 : 0;   // (the lookups may need the exact sum beyond the table: header flag 4)
    }
  }
  const int32_t j0 = ch * kTcChain;
#ifdef PROM_TRACE
  if (tid == 0) {
    tq[1] = wall_clock64();
    tq[5] = (unsigned long long)ch | ((unsigned long long)pt << 8) | ((unsigned long long)o << 16);
    tq[6] = (unsigned long long)(uint32_t)L;
    tq[2] = tq[3] = tq[4] = tq[1];
  }
#endif
  if (ch > 0 && j0 >= L) return;   // (chain 0 always runs: the moments and the header)
  // 2. this part's chords at this chain's nodes (and, chain 0, the moments); thread (k, g): node k, chords
  // c_lo + g + 16 m from LDS (the 16 threads of a group read the same entry: a broadcast)
  const int k = tid & 15, g = tid >> 4;
  double acc[kTcChain] = {0.0, 0.0, 0.0, 0.0};
  double mom = 0.0;
  const bool do_tab = fin && j0 < L;
  const double inv_fs = 1.0 / fs;
  const double inv_nmax = fin ? 1.0 / nmax : 0.0;
  // node k of octave j0: q_k = 2^(j0 - 7 + v_k), v_k = (u_k + 1) / 2, u_k = cos(pi (k + 1/2) / 16);
  // y = N q_k / N_max (-256 / ln2)
  const double sk = ldexp(tcc[kTcD * kTcD + k], j0 + kTcExpEps) * inv_nmax * kM256Ln2;
  __syncthreads();   // etab
  if (fin) {
    auto chord = [&](int32_t c) -> double2 {
      if (in_lds) return spart[c - c_lo];
      return fl[c] == 0 ? make_double2(fout[c], nc[c]) : make_double2(0.0, 0.0);
    };
    if (do_tab) {
      // kTcIlp chords per iteration (independent LDS reads and exps: one wave per SIMD here, so the chains'
      // latency is hidden only by the thread's own overlap; a chord past c_hi is the zero entry).  The adds keep
      // the chord order c, c + 16, c + 32, ... of a one-chord loop
      constexpr int kTcIlp = PROM_TC_ILP;
      for (int32_t c = c_lo + g; c < c_hi; c += kTcIlp * (kTcB2 / 16)) {
        double F[kTcIlp], e[kTcIlp];
#pragma unroll
        for (int u = 0; u < kTcIlp; ++u) {
          const int32_t cu = c + u * (kTcB2 / 16);
          const double2 f = cu < c_hi ? chord(cu) : make_double2(0.0, 0.0);
          e[u] = exp256(f.y * sk, etab);
          F[u] = f.x * inv_fs;
        }
#pragma unroll
        for (int u = 0; u < kTcIlp; ++u) acc[0] = __builtin_fma(F[u], e[u], acc[0]);
#pragma unroll
        for (int m = 1; m < kTcChain; ++m) {
#pragma unroll
          for (int u = 0; u < kTcIlp; ++u) {
            e[u] = e[u] * e[u];
            acc[m] = __builtin_fma(F[u], e[u], acc[m]);
          }
        }
      }
    }
    if (ch == 0 && k < 6) {
      // tail moments sum F n^e (e = k)
      // (four chords per iteration, added in chord order)
      for (int32_t c = c_lo + g; c < c_hi; c += 4 * (kTcB2 / 16)) {
        double n[4], pw[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int32_t cu = c + u * (kTcB2 / 16);
          const double2 fn = cu < c_hi ? chord(cu) : make_double2(0.0, 0.0);
          n[u] = fn.y * inv_nmax;
          pw[u] = fn.x * inv_fs;
        }
        for (int e2 = 0; e2 < k; ++e2) {
#pragma unroll
          for (int u = 0; u < 4; ++u) pw[u] *= n[u];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) mom += pw[u];
      }
    }
  }
  // (tcp: the part's transparent F_out sum rides in the moments row, slot 6 -- summed over the parts in order)
  if (tcp && ch == 0 && k == 6 && g == 0) mom = ts;
#ifdef PROM_TRACE
  if (lane == 0) {
    double x = acc[0] + mom;
    asm volatile("" : "+v"(x));
    atomicMax(&s_tmax[1], wall_clock64());
  }
#endif
  // fold the 16 groups: across the 4 rows of a wave (butterfly: every row the same sum), then the waves in LDS
#pragma unroll
  for (int m = 0; m < kTcChain; ++m) {
    acc[m] += __shfl_xor(acc[m], 16, 64);
    acc[m] += __shfl_xor(acc[m], 32, 64);
  }
  mom += __shfl_xor(mom, 16, 64);
  mom += __shfl_xor(mom, 32, 64);
  if (lane < 16) {
#pragma unroll
    for (int m = 0; m < kTcChain; ++m) red[wid][m][lane] = acc[m];
    red[wid][kTcChain][lane] = mom;
  }
  __syncthreads();
#ifdef PROM_TRACE
  if (tid == 0) { tq[7] = s_tmax[0]; tq[2] = s_tmax[1]; }
#endif
  const int32_t item = o * n_ch + ch;
  double* pp = part + (int64_t)item * kTcPartMax * kTcPartVals;
  // the workgroup's sums, waves in order
  double v = 0.0;
  if (tid < (kTcChain + 1) * kTcD) {
    const int m = tid >> 4, kk = tid & 15;
    v = red[0][m][kk];
#pragma unroll
    for (int w = 1; w < NW; ++w) v += red[w][m][kk];
  }
  if (n_parts == 1) {
    // every chord in this workgroup: no hand-off
    if (tid < (kTcChain + 1) * kTcD) sf[tid >> 4][tid & 15] = v;
#ifdef PROM_TRACE
    if (tid == 0) {
      tq[3] = tq[4] = wall_clock64();
      tq[6] |= 1ull << 16;
    }
#endif
  } else {
    // hand-off to the last part of this (phase, chain) (MI355X_MICROARCH.md, inter-workgroup visibility, first
    // row of the sc1 table): write-through (sc1) stores, every storing wave's vmcnt(0), a barrier, one agent-scope
    // atomic add per workgroup; the workgroup whose add comes last reads with sc1 loads after a barrier.  This is
    // the guide's measured sc1 form (global_store_dwordx2 sc1 / global_atomic_add / global_load_dwordx2 sc1 in the
    // ISA), used in place of an agent-scope release/acquire pair: the release fence is a buffer_wbl2 sc1 of the
    // whole XCD L2 (1.7 us clean, ~6.5 us with other runs' R rows dirty in it), per workgroup and run
    if (tid < (kTcChain + 1) * kTcD)
      __hip_atomic_store(&pp[pt * kTcPartVals + tid], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const int32_t prev = __hip_atomic_fetch_add(&cnt[item], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = prev == n_parts - 1 ? 1 : 0;
      // ready for the next run of this slot (a later launch: the kernel boundary orders it)
      if (s_last) __hip_atomic_store(&cnt[item], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
#ifdef PROM_TRACE
    if (tid == 0) {
      tq[3] = tq[4] = wall_clock64();
      tq[6] |= (unsigned long long)s_last << 16;
    }
#endif
    if (!s_last) return;
    if (tid < (kTcChain + 1) * kTcD) {
      // every part's value loaded first (independent loads in flight together), then added in part order
      double pv[kTcPartMax];
#pragma unroll
      for (int q = 0; q < kTcPartMax; ++q)
        pv[q] = q < n_parts ? __hip_atomic_load(&pp[q * kTcPartVals + tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
      double sv = 0.0;
#pragma unroll
      for (int q = 0; q < kTcPartMax; ++q)
        if (q < n_parts) sv += pv[q];
      sf[tid >> 4][tid & 15] = sv;
    }
  }  __syncthreads();
  if (tid < kTcChain * kTcD) {
    const int m = tid >> 4, kk = tid & 15;
    if (do_tab && j0 + m < L) {
      double c = 0.0;
#pragma unroll
      for (int jj = 0; jj < kTcD; ++jj) c = __builtin_fma(sf[m][jj], tcc[kk * kTcD + jj], c);
      tab[((int64_t)o * lg + j0 + m) * kTcD + kk] = c;
    }
  }
  if (ch == 0 && tid == 0) {
    // t_e = (-1)^e m_e / e!
    double t[6];
#pragma unroll
    for (int e = 0; e < 6; ++e) t[e] = fin ? sf[kTcChain][e] : 0.0;
    t[1] = -t[1];
    t[2] = t[2] / 2.0;
    t[3] = -t[3] / 6.0;
    t[4] = t[4] / 24.0;
    t[5] = -t[5] / 120.0;
    double* h = hdr + (int64_t)o * kTcHdr;
    h[kTcHNmax] = nmax;
    h[kTcHTfrac] = (tcp ? sf[kTcChain][6] : ts) / fs;
    h[kTcHFsum] = fs;
#pragma unroll
    for (int e = 0; e < 6; ++e) h[kTcHT0 + e] = t[e];
    h[kTcHL] = (double)L;
    h[kTcHFlags] = (double)(top_opaque | (nnf ? 2 : 0) | trunc);
    h[kTcHNact] = (double)nact;
    if (counts) {
      int32_t* cn = counts + o * kCnt;
      cn[0] = nact; cn[1] = ntr; cn[2] = nbl; cn[3] = nnf;
      cn[4] = nact; cn[5] = 0; cn[6] = 0; cn[7] = L;
    }
  }
  if (evals && tid == 0 && do_tab)
    atomicAdd(&evals[item & 63], (unsigned long long)nact * kTcD * (L - j0 < kTcChain ? L - j0 : kTcChain));
#ifdef PROM_TRACE
  if (tid == 0) tq[4] = wall_clock64();
#endif
}

// ---- sigma lookups + transmission curves -> R --------------------------------------------------------------
// The lookups are k_sigma_poly's (prom_sigma.hip): one workgroup per (256-wavelength block, R rows), per species
// the block's table slice staged in LDS ({x_k, x_{k+1}}, {10^y_k, ln10 slope_k}), one record per lookup when the
// slice's linear guess is numpy's bracket (kind & 4), the degree-D Taylor e^a; oversize blocks first, reading
// 32-byte records from the global table.  NT = R target rows with orbital Doppler shift, NT = 1 without (UNI:
// the R phases of the workgroup share one Y per wavelength).  Then each (phase, wavelength): R = T_o(Y).
// (build macro PROM_TC_WPE: pin the lookup kernel's waves per SIMD, for occupancy sweeps)
#ifndef PROM_TC_FG
#define PROM_TC_FG 2    // rows per group of global-record lookups in k_sigma_tc's front / directory paths
#endif
#ifndef PROM_TC_LGN
#define PROM_TC_LGN 4   // (its group size)
#endif
#ifndef PROM_TC_LG4
#define PROM_TC_LG4 1   // 1: k_sigma_tc's LDS lookups in groups of 4 rows (register pressure; A/B)
#endif
#ifdef PROM_TC_WPE
#define PROM_TC_ATTR __attribute__((amdgpu_waves_per_eu(PROM_TC_WPE, PROM_TC_WPE)))
#else
#define PROM_TC_ATTR
#endif
template <int NSIG, int D, bool MG, int R, bool UNI>
__global__ void __launch_bounds__(kBlock) PROM_TC_ATTR k_sigma_tc(const SigTabs4 tabv, const PolyCoef pc, const double* __restrict__ wav,
                                                     int64_t n_wav, int32_t n_rows, const SigSeg* __restrict__ seg,
                                                     const SigSeg* __restrict__ seg4, const int32_t* __restrict__ sdir,
                                                     const int32_t* __restrict__ fb, int32_t n_fb, int32_t n_blk,
                                                     int32_t n_rc, int32_t rf, const TcArgs ta) {
  static_assert(R == 1 || R == 2 || R == 4 || R == 8 || R == 16, "1 to 16 rows per workgroup");
  constexpr int NT = UNI ? 1 : R;
  // every species' slice staged at once (one load round, one barrier): per species the nodes x_k (m + 1 of them)
  // and the records' {(chi) E_k, slope_k} (24 bytes a record: four 3-species workgroups per CU)
  constexpr int CAP = tc_slice_cap(NSIG);   // (nodes per species' slice, SigSeg kind & 64)
  constexpr int SXN = CAP + 2;              // (x_0 .. x_m, padded to 16 bytes)
  __shared__ double2 ssel[(D > 0 && NT > 1) ? NSIG * CAP : 1];
  __shared__ double ssx[(D > 0 && NT > 1) ? NSIG * SXN : 1];
  const int tid = threadIdx.x;
  const int32_t RF = rf;
  const int64_t n_fb8 = ((int64_t)n_fb + 7) / 8 * 8, n_front = n_fb8 * ((n_rows + RF - 1) / RF);
  int64_t bid = blockIdx.x, wb;
  int32_t r0, rcap = R;
  bool lds_ok = true;
  if (bid < n_front) {
    const int64_t i = bid % n_fb8;
    if (i >= n_fb) return;
    wb = fb[i];
    r0 = (int32_t)(bid / n_fb8) * RF;
    rcap = RF;
    lds_ok = false;
  } else {
    bid -= n_front;
    const int64_t grp = bid / (8 * n_rc), rem = bid % (8 * n_rc);
    wb = grp * 8 + rem % 8;
    r0 = (int32_t)(rem / 8) * R;
    if (wb >= n_blk) return;
    if constexpr (NT == 1 || D == 0) {
      // one target row (one phase, or phases sharing one Doppler factor): no LDS slices -- each lane reads its
      // own 32-byte record from the global table, adjacent wavelengths' records adjacent (coalesced), no
      // barriers; every block here (the launcher passes no front)
      lds_ok = false;
    } else {
#pragma unroll
      for (int s = 0; s < NSIG; ++s) lds_ok = lds_ok && (seg[wb * NSIG + s].kind & 64) != 0;
      if (!lds_ok) return;   // (a front workgroup's)
    }
  }
  // the block's segments, every species at once
  SigSeg sgs[NSIG];
#pragma unroll
  for (int s = 0; s < NSIG; ++s) sgs[s] = seg[wb * NSIG + s];
  // the rows' curve headers, staged with the slices (read after the lookups: no load round at the end)
  __shared__ double shdr[R * kTcHdr];
  if (tid < R * kTcHdr) {
    const int32_t rr = r0 + tid / kTcHdr;
    shdr[tid] = ta.hdr[(int64_t)(rr < n_rows ? rr : n_rows - 1) * kTcHdr + tid % kTcHdr];
  }
  const int32_t rlim = r0 + rcap < n_rows ? r0 + rcap : n_rows;
  rcap = rlim - r0;
#ifdef PROM_TRACE
  const unsigned long long tr_t0 = wall_clock64();
#endif
  const int64_t w = wb * kBlock + tid;
  const bool live = w < n_wav;
  const double lam = wav[live ? w : n_wav - 1];
  // the rows' targets, once: every species of the effective absorber belongs to one density scenario (species
  // merging) or there is one species, so they share the Doppler factors
  double tt[NT];
#pragma unroll
  for (int r = 0; r < NT; ++r) tt[r] = tabv.t[0].shift[r0 + r < n_rows ? r0 + r : n_rows - 1] * lam;
  // merged: acc = sum_s fl(chi_s E_k) e^a over the species, minus choff = sum_s fl(chi_s offset_s) once at the
  // end (the same roundings: where every sigma_s is at the table floor, E_k = offset and a = 0, Y is exactly 0)
  double acc[NT];
#pragma unroll
  for (int r = 0; r < NT; ++r) acc[r] = 0.0;
  double choff = 0.0;
  if constexpr (D > 0 && NT > 1) {
    if (lds_ok) {
      // each thread: records tid, tid + 256, ... of every species' slice (m <= CAP), all loads in flight before the
      // first LDS write
      constexpr int NQ = (CAP + kBlock - 1) / kBlock;
      double4 q[NSIG][NQ];
#pragma unroll
      for (int s = 0; s < NSIG; ++s) {
        const double4* __restrict__ rr = tabv.t[s].rec + sgs[s].lo;
#pragma unroll
        for (int j = 0; j < NQ; ++j) q[s][j] = rr[tid + j * kBlock < sgs[s].m ? tid + j * kBlock : 0];
      }
#pragma unroll
      for (int s = 0; s < NSIG; ++s) {
        const double chi = tabv.t[s].chi;
        double* sx = ssx + s * SXN;
        double2* sel = ssel + s * CAP;
        const int32_t m = sgs[s].m;
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
          const int32_t i = tid + j * kBlock;
          if (i < m) {
            sx[i] = q[s][j].x;
            sel[i] = make_double2(MG ? chi * q[s][j].y : q[s][j].y, q[s][j].z);
            if (i == m - 1) sx[m] = q[s][j].w;   // the last record's upper node
          }
        }
      }
      __syncthreads();
    }
  }
  if (!lds_ok) __syncthreads();   // (shdr)
#pragma unroll
  for (int s = 0; s < NSIG; ++s) {
    const SigTabDev& tb = tabv.t[s];
    const SigSeg& sg = sgs[s];
    if constexpr (D == 0) {
      // tables too coarse for a degree-14 e^a polynomial: numpy.interp + exp10 per target (sigma_seg: the
      // block's verified guess into the global x / f arrays), bit for bit the per-target lookups
#pragma unroll
      for (int r = 0; r < NT; ++r) {
        const double v = sigma_seg(tt[r], tb, sg);
        if constexpr (MG) acc[r] += tb.chi * v;
        else acc[r] = v;
      }
      continue;
    }
    const double off = tb.offset, chi = tb.chi;
    if constexpr (MG) choff += chi * off;
    const bool exact = (sg.kind & 4) != 0;
    // v = (chi) E_k e^a: merged, accumulated; one species, sigma = E_k e^a - offset
    auto emit = [&](int r, double ce, double p) {
      if constexpr (MG) acc[r] = __builtin_fma(ce, p, acc[r]);
      else acc[r] = __builtin_fma(ce, p, -off);
    };
    const int32_t ncap = UNI ? 1 : rcap;
    if (!lds_ok) {
      // a block without a guess may have one per wavefront (kind & 8: the wave's own slice, global records)
      SigSeg sgw = sg;
      if ((sg.kind & 3) == 0 && (sg.kind & 32)) {
        // a bucket directory over the slice (kind & 32: seg4[pad] = {slice lo, buckets + 1, its offset in sdir,
        // the linear map to buckets}): the bucket's bracket, verified on the host within one node of numpy's
        constexpr int G = NT < PROM_TC_FG ? NT : PROM_TC_FG;
        const SigSeg dg = seg4[sg.pad];
        const int32_t* __restrict__ dv = sdir + dg.pad;
        const double4* __restrict__ rr = tb.rec + dg.lo;
#pragma unroll
        for (int r0g = 0; r0g < NT; r0g += G) {
          if (r0g >= ncap) break;
          int32_t gg[G];
          double4 q[G];
#pragma unroll
          for (int jj = 0; jj < G; ++jj) gg[jj] = dv[seg_guess(tt[r0g + jj], dg.xs, dg.inv, dg.m)];
#pragma unroll
          for (int jj = 0; jj < G; ++jj) q[jj] = rr[gg[jj]];
#pragma unroll
          for (int jj = 0; jj < G; ++jj) {
            const double t = tt[r0g + jj];
            const int32_t k = t < q[jj].x ? gg[jj] - 1 : (t >= q[jj].w ? gg[jj] + 1 : gg[jj]);
            if (k != gg[jj]) q[jj] = rr[k];
          }
#pragma unroll
          for (int jj = 0; jj < G; ++jj)
            emit(r0g + jj, MG ? chi * q[jj].y : q[jj].y, exp_taylor<D>(q[jj].z * (tt[r0g + jj] - q[jj].x), pc));
        }
        continue;
      }
      if ((sg.kind & 3) == 0 && (sg.kind & 8)) {
        const SigSeg sub = seg4[((int64_t)wb * NSIG + s) * 4 + (tid >> 6)];
        if (sub.m > 0) sgw = sub;
      }
      if ((sgw.kind & 3) > 0) {
        const bool exact = (sgw.kind & 4) != 0;
        constexpr int G = NT < PROM_TC_FG ? NT : PROM_TC_FG;
        const double4* __restrict__ rr = tb.rec + sgw.lo;
#pragma unroll
        for (int r0g = 0; r0g < NT; r0g += G) {
          if (r0g >= ncap) break;
          double4 q[G];
#pragma unroll
          for (int jj = 0; jj < G; ++jj) q[jj] = rr[seg_guess(tt[r0g + jj], sgw.xs, sgw.inv, sgw.m)];
          if (!exact) {
#pragma unroll
            for (int jj = 0; jj < G; ++jj) {
              const double t = tt[r0g + jj];
              const int32_t g = seg_guess(t, sgw.xs, sgw.inv, sgw.m);
              const int32_t k = t < q[jj].x ? g - 1 : (t >= q[jj].w ? g + 1 : g);
              if (k != g) q[jj] = rr[k];
            }
          }
#pragma unroll
          for (int jj = 0; jj < G; ++jj)
            emit(r0g + jj, MG ? chi * q[jj].y : q[jj].y, exp_taylor<D>(q[jj].z * (tt[r0g + jj] - q[jj].x), pc));
        }
      } else {
#pragma unroll
        for (int r = 0; r < NT; ++r) {
          if (r >= ncap) continue;
          const double v = sigma_poly_of(tt[r], tb, pc, D);
          if constexpr (MG) acc[r] = __builtin_fma(chi, v + off, acc[r]);   // (sigma + offset = E_k e^a)
          else acc[r] = v;
        }
      }
    } else if constexpr (D > 0 && NT > 1) {
      const double* sx = ssx + s * SXN;
      const double2* sel = ssel + s * CAP;
      auto lds_rows = [&](auto guard) {
        constexpr bool GD = decltype(guard)::value;
        constexpr int LG = PROM_TC_LG4 ? (NT < PROM_TC_LGN ? NT : PROM_TC_LGN) : NT;   // rows per group of lookups in flight
#pragma unroll
        for (int r0g = 0; r0g < NT; r0g += LG) {
          double xk[LG];
          double2 el[LG];
#pragma unroll
          for (int rr = 0; rr < LG; ++rr) {
            const int r = r0g + rr;
            if (GD && r >= ncap) break;
            const int32_t g = seg_guess(tt[r], sg.xs, sg.inv, sg.m);
            if (exact) {
              xk[rr] = sx[g];
              el[rr] = sel[g];
            } else {
              const double2 xx = make_double2(sx[g], sx[g + 1]);
              const int32_t k = tt[r] < xx.x ? g - 1 : (tt[r] >= xx.y ? g + 1 : g);
              xk[rr] = sx[k];
              el[rr] = sel[k];
            }
          }
#pragma unroll
          for (int rr = 0; rr < LG; ++rr) {
            const int r = r0g + rr;
            if (GD && r >= ncap) break;
            emit(r, el[rr].x, exp_taylor<D>(el[rr].y * (tt[r] - xk[rr]), pc));
          }
        }
      };
      if (ncap >= NT) lds_rows(std::false_type{});
      else lds_rows(std::true_type{});
    }
  }
  if constexpr (MG && D > 0) {
#pragma unroll
    for (int r = 0; r < NT; ++r) acc[r] -= choff;
  }
  // R = T_o(Y) per (phase, wavelength)
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (r >= rcap) break;
    const int32_t o = r0 + r;
    const double Y = acc[UNI ? 0 : r];
    const double* h = shdr + r * kTcHdr;
    double v;
    if (!((int32_t)h[kTcHFlags] & 2)) {
      v = tc_eval(Y, h, ta.tab + (int64_t)o * ta.lg * kTcD, ta.flags + (int64_t)o * ta.n_pr,
                  ta.ncol + (int64_t)o * ta.n_pr, ta.fout, ta.n_pr, ta.evals);
    } else {
      // non-finite column densities: the reference's chord order with ocml exp.  Merged species: the
      // reference's sum_s (N chi_s) sigma_s is NaN for an infinite N wherever some chi_s sigma_s is not > 0
      bool zr = false;
      if constexpr (MG) {
#pragma unroll
        for (int s = 0; s < NSIG; ++s) {
          const SigTabDev& tb = tabv.t[s];
          const double sv = D == 0 ? sigma_seg(tb.shift[o] * lam, tb, seg[wb * NSIG + s])
                                   : sigma_seg_poly(tb.shift[o] * lam, tb, seg[wb * NSIG + s], pc, D);
          zr = zr || !(tb.chi * sv > 0.0);
        }
      }
      const int32_t* fl = ta.flags + (int64_t)o * ta.n_pr;
      const double* nc = ta.ncol + (int64_t)o * ta.n_pr;
      double a = 0.0;
      for (int32_t c = 0; c < ta.n_pr; ++c) {
        if (fl[c] != 0) continue;
        const double N = nc[c];
        double tau = N * Y;
        if (zr && !__builtin_isfinite(N)) tau = __builtin_nan("");
        a = a + ta.fout[c] * exp(-tau);
      }
      const double fs = h[kTcHFsum];
      v = (a + h[kTcHTfrac] * fs) / fs;
    }
    if (live) ta.R[(int64_t)o * n_wav + w] = v;
  }
#ifdef PROM_TRACE
  // per workgroup (tools/trace_sigma.py): start, end (wall clock, 10 ns), block | lds << 32 | front << 33,
  // first row | species kinds << 32 | largest slice << 44
  if (threadIdx.x == 0 && blockIdx.x < (1u << 18)) {
    unsigned long long* tp = g_trace + 4ull * blockIdx.x;
    tp[0] = tr_t0;
    tp[1] = wall_clock64();
    tp[2] = (unsigned long long)wb | ((unsigned long long)lds_ok << 32) | ((unsigned long long)(blockIdx.x < n_front) << 33);
    unsigned long long kinds = 0;
    int32_t mmax = 0;
    for (int s = 0; s < NSIG; ++s) {
      const int32_t kd = seg[wb * NSIG + s].kind;   // (3: no linear guess, a bucket directory)
      kinds |= (unsigned long long)((kd & 3) == 0 && (kd & 32) ? 3 : (kd & 7)) << (3 * s);
      mmax = seg[wb * NSIG + s].m > mmax ? seg[wb * NSIG + s].m : mmax;
    }
    tp[3] = (unsigned long long)(uint32_t)r0 | (kinds << 32) | ((unsigned long long)(mmax > 65535 ? 65535 : mmax) << 44);
  }
#endif
}

#ifdef PROM_TRACE
extern "C" int32_t prom_tc_trace_read(unsigned long long* out, int32_t n, int32_t clear) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trace), sizeof(unsigned long long) * n) != hipSuccess) return -1;
  if (clear) {
    static unsigned long long zeros[1 << 20];
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_trace), zeros, sizeof(zeros)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

bool launch_tcurve(hipStream_t s, TransitDev& tr, RunSlot& rs, int32_t nsig, bool msp, hipEvent_t ev_sig0,
                   hipEvent_t ev_sig1, hipEvent_t ev_tb0, hipEvent_t ev_tb1) {
  const int32_t lg = tr.tc_lg;
  unsigned long long* evals = tr.count_evals ? rs.evals.as<unsigned long long>() : nullptr;
  const int32_t n_ch = (lg + kTcChain - 1) / kTcChain;
  const int32_t n_parts = tr.tc_parts;
  // (k_columns8 wrote the phase partials when n_pr % 32 == 0: launch_transit's col_tcp rule)
  const TcPart* pp = tr.tc_pp_ok ? rs.tc_pp.as<TcPart>() : nullptr;
  hipExtLaunchKernelGGL(k_tc_build, dim3((unsigned)n_ch, (unsigned)n_parts, (unsigned)tr.n_orb), dim3(kTcB2), 0, s,
                        ev_tb0, ev_tb1, 0, rs.flags.as<int32_t>(), tr.cfout.as<double>(), rs.ncol.as<double>(), tr.n_pr,
                        n_parts, tr.tc_ybound, lg, tr.tc_const.as<double>(), rs.tc_hdr.as<double>(), rs.tc_tab.as<double>(), rs.tc_part.as<double>(),
                        rs.tc_cnt.as<int32_t>(), rs.counts.as<int32_t>(), evals, pp, tr.tc_fsum);
  PROM_HIP(hipGetLastError());
  TcArgs ta{};
  ta.hdr = rs.tc_hdr.as<double>();
  ta.tab = rs.tc_tab.as<double>();
  ta.flags = rs.flags.as<int32_t>();
  ta.ncol = rs.ncol.as<double>();
  ta.fout = tr.cfout.as<double>();
  ta.R = rs.R.as<double>();
  ta.evals = evals;
  ta.lg = lg;
  ta.n_pr = tr.n_pr;
  const bool uni = tr.uniform_shift;
  const int32_t n_rows = tr.n_orb;
  const int64_t n_wav = tr.n_wav;
  const int32_t n_blk = (int32_t)grid_for(n_wav);
  // rows per workgroup: 8 (every species' slice staged once for 8 phases; one species with orbital Doppler shift
  // took 4 until round 5: C4x10 0.077 -> 0.064 ms per pipelined step with 8, C4 0.0116 -> 0.0111, profiles/r05h_*),
  // never more than the problem's (instantiated: 8 rows with one shared target; 1, 4 or 8 with orbital Doppler
  // shift -- the guarded copy of the lookups covers workgroups with fewer rows).  PROM_TC_R1 (profiling, read once):
  // 4 rows for one species
  const int deg = tr.sig_deg;
  static const int r1_env = [] { const char* e = std::getenv("PROM_TC_R1"); return e ? std::atoi(e) : 0; }();
  const int Rmax = (nsig >= 2 || uni) ? 8 : (r1_env == 4 ? 4 : 8);
  const int R = (uni || deg == 0) ? 8 : (n_rows == 1 ? 1 : Rmax);
  const int32_t n_rc = (n_rows + R - 1) / R;
  // front workgroups (oversize blocks): R / 2 rows for one species with fewer than 16384 (block, row) pairs of
  // them (profiles/r03_sigma_rf_sweep.txt), or for several species when some block has neither a linear guess
  // nor a directory (its slow lookups spread over more workgroups); else all R (C3 with every block guessed:
  // 34.5 -> 32.6 us, profiles/r04t_front_rows_sweep.txt); one shared target: all R
  int RF = R;
  if (!uni && R >= 2 && ((nsig >= 2 && tr.sig_noguess > 0) || (nsig == 1 && (int64_t)tr.n_sig_fb_tc * n_rows < 16384)))
    RF = R / 2;
  // PROM_TC_RF (profiling): rows per front workgroup, 1 .. R (read once)
  static const int rf_env = [] { const char* e = std::getenv("PROM_TC_RF"); return e ? std::atoi(e) : 0; }();
  if (rf_env >= 1 && rf_env <= R) RF = rf_env;
  // one target row (NT == 1: no Doppler shift between the phases, or one phase): every block reads the global
  // records directly, no front of oversize blocks
  // (deg == 0: the exp10 lookups read the global arrays in every block -- k_sigma_tc's main grid takes the oversize
  // blocks too, so no front: a front would look them up and write their R rows a second time)
  const bool direct = uni || R == 1 || deg == 0;
  const int32_t n_fb = direct ? 0 : tr.n_sig_fb_tc;
  const int64_t n_front = (int64_t)((n_fb + 7) / 8) * 8 * ((n_rows + RF - 1) / RF);
  const unsigned nb = (unsigned)(n_front + (n_fb >= n_blk ? 0 : (int64_t)((n_blk + 7) / 8) * 8 * n_rc));
  const PolyCoef& pc = poly_coef();
  const SigTabs4& tabv = tr.sigtab_v;
  const double* wav = tr.wav.as<double>();
  const SigSeg* seg = tr.sig_seg.as<SigSeg>();
  const SigSeg* seg4 = tr.sig_seg4.as<SigSeg>();
  const int32_t* sdir = tr.sig_dir.as<int32_t>();
  const int32_t* fb = tr.sig_fb_tc.as<int32_t>();
  PROM_REQUIRE(msp || nsig == 1, "transmission curves: one effective absorber only");
  if (tr.tw_ok && !uni && deg > 0 && n_rows >= 2 && tr.n_tw > 0) {
    // target windows (k_sigma_tw, prom_tw.hip)
    launch_sigma_tw(s, tr, nsig, deg, ta, ev_sig0, ev_sig1);
    return true;
  }
#define PROM_TCK(NS, DG, MGV, RV, UV)                                                                         \
  hipExtLaunchKernelGGL((k_sigma_tc<NS, DG, MGV, RV, UV>), dim3(nb), dim3(kBlock), 0, s, ev_sig0, ev_sig1, 0, tabv, \
                        pc, wav, n_wav, n_rows, seg, seg4, sdir, fb, n_fb, n_blk, n_rc, RF, ta)
#define PROM_TCR(NS, DG, MGV)                                       \
  do {                                                              \
    if (uni) PROM_TCK(NS, DG, MGV, 8, true);                        \
    else if (R == 1) PROM_TCK(NS, DG, MGV, 1, false);               \
    else if ((NS) == 1 && R == 4) PROM_TCK(NS, DG, MGV, 4, false);   \
    else PROM_TCK(NS, DG, MGV, 8, false);                           \
  } while (0)
  // degree 8 covers every table with amax <= 0.07 (the high-resolution configs); 14 the rest (coarse tables)
#define PROM_TCD(NS, MGV)                                                          \
  if (deg == 0) { if (uni) PROM_TCK(NS, 0, MGV, 8, true); else PROM_TCK(NS, 0, MGV, 8, false); } \
  else if (deg <= 8) PROM_TCR(NS, 8, MGV);                                       \
  else PROM_TCR(NS, 14, MGV);
#ifdef PROM_TC_DEV_ONE
  // (development builds: the C3 instantiations only, for quick resource-usage checks)
  PROM_TCR(3, 8, true);
#else
  switch (nsig) {
    case 1: PROM_TCD(1, false) break;
    case 2: PROM_TCD(2, true) break;
    case 3: PROM_TCD(3, true) break;
    default: PROM_TCD(4, true) break;
  }
#endif
#undef PROM_TCD
#undef PROM_TCR
#undef PROM_TCK
  PROM_HIP(hipGetLastError());
  return false;
}

}  // namespace prom
