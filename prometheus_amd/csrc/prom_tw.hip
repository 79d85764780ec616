// k_sigma_tw: the Doppler-shifted cross-section lookups and transmission curves over target windows.
#include "prom_tc.h"

namespace prom {

// ---- sigma lookups + transmission curves over target windows (the default with orbital Doppler shift) ----
// The targets t = shift_o lambda_w of all rows, not the wavelengths, are cut into windows (host: prom_window.hip):
// window b holds, per row o, the contiguous wavelengths w in [W[b][o], W[b+1][o]) whose targets fall in the
// window's target interval (at most a few hundred per row).  Per species the table nodes those targets reach are
// one slice, staged once per window for every row: no Doppler-spread overlap between neighbouring windows' slices
// and no second workgroup staging the same slice for other rows.  The wavelengths the rows read, [lw0, lw1), are
// staged with them: the item loop then issues no vector load, only its stores (on gfx9 a load's vmcnt wait also
// waits for every earlier store: a global wavelength load per item cost each item a store round trip).  Slices and
// wavelengths share kTwLds doubles of LDS (22 KB: 24 bytes a node, 8 a wavelength), carved per window by the host.
// Work items are (row, 64 wavelengths) with the row wave-uniform: its Doppler factor, curve header and coefficients
// are scalar loads.  Per species slice (SigSeg kind & 3): 1 staged, with the host-verified linear guess (one LDS
// round: x_g, x_{g+1} and the record; a second only for lanes one node off); 3 staged without a guess (a slice
// across a change of node spacing: bisection in LDS); 2 the guess into the global records (a slice larger than the
// LDS) or 0 none (targets outside the table): the window goes to the second pass.  The second pass also takes the rows
// whose curve header says non-finite columns (flag 2, the reference's chord order) or a table truncated at the host's
// octave cap (flag 4, the exact sum beyond it): numpy's bracket from the table's directory, per point.  Every path
// evaluates fl(chi E_k) e^a (or E_k e^a - offset) of numpy's bracket k, so R does not depend on the windows: bitwise
// equal to k_sigma_tc's and for any wavelength or phase shard.

template <int NSIG, int D, bool MG, int RP>
__global__ void __launch_bounds__(kBlock) k_sigma_tw(const SigTabs4 tabv, const SigTabDev* __restrict__ tabp,
                                                     const PolyCoef pc, const double* __restrict__ wav,
                                                     int64_t n_wav, int32_t n_rows, const SigSeg* __restrict__ wseg,
                                                     const int32_t* __restrict__ wrow, const int32_t* __restrict__ wlam,
                                                     int32_t n_win, const TcArgs ta,
                                                     const double* __restrict__ hdr, const double* __restrict__ shift,
                                                     const double* __restrict__ ctab, double* __restrict__ Rout) {
  // (hdr, shift, ctab, Rout: TcArgs' hdr, tabv.t[0].shift, tab and R as __restrict__ parameters -- with the kernel's
  // stores provably elsewhere, the row's header and Doppler factor become scalar loads)
  static_assert(D > 0, "polynomial lookups only (coarse tables take k_sigma_tc)");
  // LDS: [0, 2 tot) the records {(chi) E_k, L_k} (species s at 2 pad), then tot + NSIG node x's (species s at pad + s:
  // x_lo .. x_{lo+m}), then the window's wavelengths
  __shared__ double2 lds2[kTwLds / 2 + 32];   // (+ 64 doubles: the staged wavelengths' padding, read past lw1)
  double* const lds = reinterpret_cast<double*>(lds2);
  // XCD-aware: workgroup ids round-robin over the 8 XCDs; XCD x takes windows [x per, (x + 1) per) in order, so
  // neighbouring windows (whose rows read overlapping wavelengths) share an L2
  const int32_t per = (n_win + 7) >> 3;
  const int32_t b = (int32_t)(blockIdx.x & 7) * per + (int32_t)(blockIdx.x >> 3);
  if (b >= n_win) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  SigSeg sg[NSIG];
  bool wrare = false;   // (some species without a slice: second pass for the whole window)
  bool wexact = true;   // (every guess is numpy's bracket at every target of the window: k_tw_exact, kind & 4)
  bool wsearch = false; // (some staged slice without a guess, kind 3: bisection in LDS)
  int32_t tot = 0;      // staged nodes (kinds 1 and 3)
#pragma unroll
  for (int s = 0; s < NSIG; ++s) {
    sg[s] = wseg[(int64_t)b * NSIG + s];
    wrare = wrare || ((sg[s].kind & 3) != 1 && (sg[s].kind & 3) != 3);
    wsearch = wsearch || (sg[s].kind & 3) == 3;
    wexact = wexact && (sg[s].kind & 4) != 0;
    if (sg[s].kind & 1) tot = sg[s].pad + sg[s].m > tot ? sg[s].pad + sg[s].m : tot;
  }
  const int32_t lw0 = wlam[2 * b], nlam = wlam[2 * b + 1] - lw0;   // (nlam = 0: wavelengths from global memory)
  double2* const sel = lds2;
  double* const sx = lds + 2 * tot;
  double* const slam = sx + tot + NSIG;
  // stage the slices (pool entry i belongs to the species whose [pad, pad + m) holds it) and the wavelengths; every
  // load issued before the first LDS write
  {
    constexpr int NQ = (kTwLds / 3 + kBlock - 1) / kBlock;
    constexpr int NL = (kTwLamCap + kBlock - 1) / kBlock;
    double lq[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int32_t i = tid + j * kBlock;
      lq[j] = i < nlam ? wav[lw0 + i] : 0.0;
    }
    double4 q[NQ];
    int sp[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int32_t i = tid + j * kBlock;
      sp[j] = -1;
#pragma unroll
      for (int s = 0; s < NSIG; ++s)
        if ((sg[s].kind & 1) && i >= sg[s].pad && i < sg[s].pad + sg[s].m) sp[j] = s;
      int32_t gi = 0;
      const double4* __restrict__ rr = tabv.t[0].rec;
#pragma unroll
      for (int s = 0; s < NSIG; ++s)
        if (sp[j] == s) {
          gi = sg[s].lo + (i - sg[s].pad);
          rr = tabv.t[s].rec;
        }
      q[j] = i < tot ? rr[gi] : make_double4(0.0, 0.0, 0.0, 0.0);
    }
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int32_t i = tid + j * kBlock;
#pragma unroll
      for (int s = 0; s < NSIG; ++s) {
        if (sp[j] != s) continue;
        sx[i + s] = q[j].x;
        sel[i] = make_double2(MG ? tabv.t[s].chi * q[j].y : q[j].y, q[j].z);
        if (i == sg[s].pad + sg[s].m - 1) sx[i + s + 1] = q[j].w;   // the slice's last upper node
      }
    }
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      const int32_t i = tid + j * kBlock;
      if (i < nlam) slam[i] = lq[j];
    }
  }
  __syncthreads();
  double choff = 0.0;
  if constexpr (MG) {
#pragma unroll
    for (int s = 0; s < NSIG; ++s) choff += tabv.t[s].chi * tabv.t[s].offset;
  }
  const int32_t* __restrict__ wa = wrow + (int64_t)b * n_rows;
  const int32_t* __restrict__ wz = wa + n_rows;
  // first pass: windows whose every species has a staged, guessed slice (kind 1), rows whose curve is complete (header
  // flags 2 and 4 clear).  Waves take whole rows (or row pairs) round robin, each row's Doppler factor and curve header
  // loaded once into scalar registers, then the rows' chunks of 64 wavelengths
  if (!wrare) {
    // per species, hoisted by hand (the compiler keeps them as per-lookup arithmetic otherwise): the slice's LDS
    // bases (lookup address = g * 8 + base), and the guess's offset and the polynomial's leading coefficient held in
    // VGPRs (a 64-bit FMA takes one scalar operand: either would be copied to VGPRs before every use)
    const double* xsb[NSIG];
    const double2* elb[NSIG];
    double xsv[NSIG];
#pragma unroll
    for (int s = 0; s < NSIG; ++s) {
      xsb[s] = sx + sg[s].pad + s;
      elb[s] = sel + sg[s].pad;
      xsv[s] = sg[s].xs;
      asm volatile("" : "+v"(xsv[s]));
    }
    double cdv = pc.c[D];
    asm volatile("" : "+v"(cdv));
    const double* lamb = slam + lane - lw0;   // (the staged wavelengths, this lane's column; 64 entries of padding)
    // NP points per lane at once: rows a and b (RP = 2: a row pair, the two rows' chunks k side by side -- two
    // independent lookup chains per lane), with each row's Doppler factor, header, table and R row in scalar registers
    struct RowS {
      const double* h;
      const double* tabo;
      double* Rrow;
      double sh;
      int32_t w0, w1;
    };
    auto row_of = [&](int32_t o) {
      RowS r;
      r.h = hdr + (int64_t)o * kTcHdr;
      r.tabo = ctab + (int64_t)o * ta.lg * kTcD;
      r.Rrow = Rout + (int64_t)o * n_wav + lane;   // (this lane's column of the row)
      r.sh = shift[o];
      r.w0 = wa[o];
      r.w1 = wz[o];
      return r;
    };
    // MODE 0: every guess exact; 1: guesses with the one-node test; 2: as 1, kind-3 slices by bisection.  c0[p]: the
    // chunk's first wavelength (stores only where c0[p] + lane < w1), lam[p] the lane's wavelength
    auto chunk = [&](const RowS* rs, auto np_tag, const int32_t* c0, const double* lam, auto mode_tag) {
      constexpr int NP = decltype(np_tag)::value;
      constexpr int MODE = decltype(mode_tag)::value;
      constexpr bool EX = MODE == 0;
      double t[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) t[p] = rs[p].sh * lam[p];
      // every species' x_g (x_{g+1}) and record in one LDS round, then, unless every guess is exact, the rare
      // one-node corrections, then the e^a polynomials.  (The guess clamps at m - 2 only: every target of the
      // window lies in the slice, so fma(t, inv, xs) > -1 and the integer conversion is >= 0, as seg_guess's)
      int32_t g[NP][NSIG];
      double x0[NP][NSIG], x1[NP][NSIG];
      double2 e[NP][NSIG];
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int s = 0; s < NSIG; ++s) {
          g[p][s] = min((int32_t)__builtin_fma(t[p], sg[s].inv, xsv[s]), sg[s].m - 2);
          x0[p][s] = xsb[s][g[p][s]];
          if constexpr (!EX) x1[p][s] = xsb[s][g[p][s] + 1];
          e[p][s] = elb[s][g[p][s]];
        }
      if constexpr (!EX) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
          for (int s = 0; s < NSIG; ++s) {
            if (MODE == 2 && (sg[s].kind & 3) == 3) {
              // numpy's bracket, the largest k <= m - 2 with x_k <= t, by bisection over the staged slice
              int32_t k = 0;
              for (int32_t st = 1 << (31 - __builtin_clz((uint32_t)(sg[s].m - 1) | 1u)); st > 0; st >>= 1)
                if (k + st <= sg[s].m - 2 && xsb[s][k + st] <= t[p]) k += st;
              x0[p][s] = xsb[s][k];
              e[p][s] = elb[s][k];
              continue;
            }
            const bool lo = t[p] < x0[p][s], hi = t[p] >= x1[p][s];   // (no short-circuit: that would chain the reads)
            if (lo | hi) {
              const int32_t k = lo ? g[p][s] - 1 : g[p][s] + 1;
              x0[p][s] = xsb[s][k];
              e[p][s] = elb[s][k];
            }
          }
      }
      double acc[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        acc[p] = 0.0;
#pragma unroll
        for (int s = 0; s < NSIG; ++s) {
          const double a = e[p][s].y * (t[p] - x0[p][s]);
          double q = __builtin_fma(cdv, a, pc.c[D - 1]);   // (exp_taylor<D>, the leading coefficient from a VGPR)
#pragma unroll
          for (int k = D - 2; k >= 0; --k) q = __builtin_fma(q, a, pc.c[k]);
          if constexpr (MG) acc[p] = __builtin_fma(e[p][s].x, q, acc[p]);
          else acc[p] = __builtin_fma(e[p][s].x, q, -tabv.t[s].offset);
        }
        if constexpr (MG) acc[p] -= choff;
      }
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const double v = tc_eval_full_s(acc[p], rs[p].h, rs[p].tabo);
        if (c0[p] + lane < rs[p].w1) rs[p].Rrow[c0[p]] = v;
      }
    };
    // the NP rows' chunks k = k0, k0 + G, ...: the wavelengths from the LDS stage, else loaded up to four chunks at a
    // time before any of them is computed (one vmcnt wait -- which also waits for the earlier stores -- per batch).  A
    // row with fewer chunks than its partner computes a clamped chunk and stores nothing
    auto rows = [&](const RowS* rs, auto np_tag, int32_t k0, int32_t G, auto mode_tag) {
      constexpr int NP = decltype(np_tag)::value;
      int32_t nch = 0;
#pragma unroll
      for (int p = 0; p < NP; ++p) nch = max(nch, (rs[p].w1 - rs[p].w0 + 63) >> 6);
      auto cfix = [&](int p, int32_t c) { return c < rs[p].w1 ? c : rs[p].w0; };   // (a clamped, computed chunk)
      if (nlam > 0) {
        for (int32_t k = k0; k < nch; k += G) {
          int32_t c0[NP];
          double lam[NP];
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            c0[p] = rs[p].w0 + 64 * k;
            lam[p] = lamb[cfix(p, c0[p])];
          }
          chunk(rs, np_tag, c0, lam, mode_tag);
        }
      } else {
        constexpr int B = 4 / NP;
        for (int32_t k = k0; k < nch; k += B * G) {
          double lam[B][NP];
#pragma unroll
          for (int j = 0; j < B; ++j)
#pragma unroll
            for (int p = 0; p < NP; ++p) {
              const int32_t w = cfix(p, rs[p].w0 + 64 * (k + j * G)) + lane;
              lam[j][p] = wav[w < rs[p].w1 ? w : rs[p].w1 - 1];
            }
#pragma unroll
          for (int j = 0; j < B; ++j) {
            if (k + j * G >= nch) break;
            int32_t c0[NP];
#pragma unroll
            for (int p = 0; p < NP; ++p) c0[p] = rs[p].w0 + 64 * (k + j * G);
            chunk(rs, np_tag, c0, lam[j], mode_tag);
          }
        }
      }
    };
    auto rows_mode = [&](const RowS* rs, auto np_tag, int32_t k0, int32_t G) {
      if (wexact) rows(rs, np_tag, k0, G, std::integral_constant<int, 0>{});
      else if (!wsearch) rows(rs, np_tag, k0, G, std::integral_constant<int, 1>{});
      else rows(rs, np_tag, k0, G, std::integral_constant<int, 2>{});
    };
    auto rare_row = [&](int32_t o) { return ((int32_t)hdr[(int64_t)o * kTcHdr + kTcHFlags] & 6) != 0; };
    if constexpr (RP == 1) {
      const int32_t G = n_rows >= 4 ? 1 : (n_rows == 1 ? 4 : 2);   // waves per row
      for (int32_t o = __builtin_amdgcn_readfirstlane(wv / G); o < n_rows; o += 4 / G) {
        if (rare_row(o)) continue;   // (second pass)
        const RowS r1[1] = {row_of(o)};
        rows_mode(r1, std::integral_constant<int, 1>{}, wv % G, G);
      }
    } else {
      // row pairs (2q, 2q + 1) round robin over the waves (G waves per pair when there are fewer than 4 pairs); a pair
      // with one row in the second pass (or past n_rows) runs its other row alone
      const int32_t P = (n_rows + 1) >> 1;
      const int32_t G = P >= 4 ? 1 : (P == 1 ? 4 : 2);
      for (int32_t q = __builtin_amdgcn_readfirstlane(wv / G); q < P; q += 4 / G) {
        const int32_t oa = 2 * q, ob = 2 * q + 1;
        const bool ra = rare_row(oa), rb = ob >= n_rows || rare_row(ob);
        if (!ra && !rb) {
          const RowS r2[2] = {row_of(oa), row_of(ob)};
          rows_mode(r2, std::integral_constant<int, 2>{}, wv % G, G);
        } else if (!ra || !rb) {
          const RowS r1[1] = {row_of(ra ? ob : oa)};
          rows_mode(r1, std::integral_constant<int, 1>{}, wv % G, G);
        }
      }
    }
  }
  // second pass: the rest (kinds 0, 2, 3, rows with header flags 2 or 4), numpy's bracket per
  // point from the table's directory; items (row o, chunk c of 64 wavelengths) to waves round robin
  auto run_pass = [&](auto pass_tag) {
    constexpr int pass = decltype(pass_tag)::value;
    // the next item of this pass at or after (o, c): its row's wavelength range, or o = n_rows
    auto next_item = [&](int32_t& o, int32_t& c, int32_t& w0, int32_t& w1) {
      o = __builtin_amdgcn_readfirstlane(o);
      c = __builtin_amdgcn_readfirstlane(c);
      while (o < n_rows) {
        const bool rare = wrare || ((int32_t)hdr[(int64_t)o * kTcHdr + kTcHFlags] & 6) != 0;
        if (rare == (pass == 1)) {
          w0 = __builtin_amdgcn_readfirstlane(wa[o]);
          w1 = __builtin_amdgcn_readfirstlane(wz[o]);
          const int32_t nch = (w1 - w0 + 63) >> 6;
          if (c < nch) return;
          c = __builtin_amdgcn_readfirstlane(c - nch);
        }
        o = __builtin_amdgcn_readfirstlane(o + 1);
      }
    };
    int32_t on = 0, cn = wv, w0n = 0, w1n = 0;
    next_item(on, cn, w0n, w1n);
    while (on < n_rows) {
      const int32_t o = __builtin_amdgcn_readfirstlane(on), w1 = __builtin_amdgcn_readfirstlane(w1n);
      const int32_t w = __builtin_amdgcn_readfirstlane(w0n + cn * 64) + lane;
      const bool live = w < w1;
      const double lam = wav[live ? w : w1 - 1];
      cn += 4;
      next_item(on, cn, w0n, w1n);
      const double t = shift[o] * lam;
      const double* h = hdr + (int64_t)o * kTcHdr;
      double acc = 0.0, v;
      {
        // second pass: numpy's bracket per point; zr (merged species, non-finite columns): some chi_s sigma_s not > 0
        bool zr = false;
#pragma unroll
        for (int s = 0; s < NSIG; ++s) {
          const SigTabDev& tb = tabp[s];   // (from memory here: the argument copy's fields would stay live in SGPRs)
          if (t >= tb.xfirst && t < tb.xlast) {
            const double4 q = tb.rec[bracket_of(t, tb)];
            const double ex = exp_taylor<D>(q.z * (t - q.x), pc);
            if constexpr (MG) {
              acc = __builtin_fma(tb.chi * q.y, ex, acc);
              zr = zr || !(tb.chi * __builtin_fma(q.y, ex, -tb.offset) > 0.0);
            } else {
              acc = __builtin_fma(q.y, ex, -tb.offset);
            }
          } else {
            const double sv = sigma_poly_of(t, tb, pc, D);   // (numpy's end rules)
            if constexpr (MG) {
              acc = __builtin_fma(tb.chi, sv + tb.offset, acc);
              zr = zr || !(tb.chi * sv > 0.0);
            } else {
              acc = sv;
            }
          }
        }
        if constexpr (MG) acc -= choff;
        const double Y = acc;
        // non-finite columns (flag 2): the reference's chord order with ocml exp (k_sigma_tc's rule); else the curve,
        // or beyond a truncated table the exact sum in chord order (tc_eval's) -- one chord loop for both
        const bool nf = ((int32_t)h[kTcHFlags] & 2) != 0;
        const double q = Y * h[kTcHNmax];
        const int32_t L = (int32_t)h[kTcHL];
        const int32_t j = q <= 1.0e300 ? tc_exponent(q) - kTcExpEps : 0x7fffffff;
        const bool beyond = !nf && q >= kTcEps && q == q && j >= L && !((int32_t)h[kTcHFlags] & 1);
        if (!nf && !beyond) {
          v = tc_eval_full(Y, h, ctab + (int64_t)o * ta.lg * kTcD);
        } else {
          const double fs = h[kTcHFsum];
          const double a = tc_chord_sum(Y, nf, zr, fs, ta.flags + (int64_t)o * ta.n_pr, ta.ncol + (int64_t)o * ta.n_pr,
                                        ta.fout, ta.n_pr);
          if (beyond && ta.evals) atomicAdd(&ta.evals[threadIdx.x & 63], (unsigned long long)(int32_t)h[kTcHNact]);
          v = nf ? (a + h[kTcHTfrac] * fs) / fs : h[kTcHTfrac] + a;
        }
      }
      if (live) Rout[(int64_t)o * n_wav + w] = v;
    }
  };
  run_pass(std::integral_constant<int, 1>{});
}

// per set (prom_transit_set, after new windows): a window's guessed slices (kind 1) are exact (kind |= 4) when every
// guess is numpy's bracket at every target the window's rows look up (k_seg_exact's test on the windows): k_sigma_tw
// then reads x_g and the record only, with no bracket test
template <int NSIG>
__global__ void __launch_bounds__(kBlock) k_tw_exact(const SigTabs4 tabv, const double* __restrict__ wav,
                                                     int32_t n_rows, SigSeg* __restrict__ wseg,
                                                     const int32_t* __restrict__ wrow) {
  const int32_t b = blockIdx.x;
  const int32_t* wa = wrow + (int64_t)b * n_rows;
  const int32_t* wz = wa + n_rows;
  __shared__ int32_t bad;
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  bool ok = true;
  for (int32_t o = 0; o < n_rows; ++o) {
    const int32_t w0 = wa[o], w1 = wz[o];
    for (int32_t w = w0 + (int32_t)threadIdx.x; w < w1; w += kBlock) {
      const double t = tabv.t[0].shift[o] * wav[w];
#pragma unroll
      for (int s = 0; s < NSIG; ++s) {
        const SigSeg sg = wseg[(int64_t)b * NSIG + s];
        if ((sg.kind & 3) != 1) continue;
        const int32_t g = seg_guess(t, sg.xs, sg.inv, sg.m);
        const double* __restrict__ X = tabv.t[s].x + sg.lo;
        int32_t a = 0, c = sg.m - 1;   // X[a] <= t < X[c]: the window's slice bounds every target
        while (c - a > 1) {
          const int32_t mid = (a + c) >> 1;
          if (X[mid] <= t) a = mid; else c = mid;
        }
        ok = ok && a == g;
      }
    }
  }
  if (!ok) bad = 1;   // (benign race: every writer stores 1)
  __syncthreads();
  if (threadIdx.x < NSIG && !bad) {
    SigSeg& sg = wseg[(int64_t)b * NSIG + threadIdx.x];
    if ((sg.kind & 3) == 1) sg.kind |= 4;
  }
}

void launch_tw_exact(hipStream_t s, TransitDev& tr, int32_t nsig) {
  if (!tr.tw_ok || tr.n_tw <= 0) return;
  SigSeg* twseg = tr.tw_seg.as<SigSeg>();
  const int32_t* twrow = tr.tw_row.as<int32_t>();
#define PROM_TWE(NS)                                                                                            \
  hipLaunchKernelGGL((k_tw_exact<NS>), dim3((unsigned)tr.n_tw), dim3(kBlock), 0, s, tr.sigtab_v, tr.wav.as<double>(), \
                     tr.n_orb, twseg, twrow)
  switch (nsig) {
    case 1: PROM_TWE(1); break;
    case 2: PROM_TWE(2); break;
    case 3: PROM_TWE(3); break;
    default: PROM_TWE(4); break;
  }
#undef PROM_TWE
  PROM_HIP(hipGetLastError());
}

void launch_sigma_tw(hipStream_t s, TransitDev& tr, int32_t nsig, int32_t deg, const TcArgs& ta, hipEvent_t ev0,
                     hipEvent_t ev1) {
  const unsigned nbw = (unsigned)(((int64_t)tr.n_tw + 7) / 8 * 8);   // one workgroup per window, XCD-interleaved ids
  const SigSeg* twseg = tr.tw_seg.as<SigSeg>();
  const int32_t* twrow = tr.tw_row.as<int32_t>();
  const int32_t* twlam = tr.tw_lam.as<int32_t>();
  const PolyCoef& pc = poly_coef();
  const SigTabs4& tabv = tr.sigtab_v;
  const SigTabDev* tabp = tr.sigtab.as<SigTabDev>();   // (the same descriptors in device memory: the second pass)
  const double* wav = tr.wav.as<double>();
  const int32_t n_rows = tr.n_orb;
  const int64_t n_wav = tr.n_wav;
  PROM_REQUIRE(deg > 0 && n_rows >= 2 && tr.n_tw > 0, "k_sigma_tw: polynomial lookups with orbital Doppler rows");
  // row pairs per wave in the first pass (two lookup chains per lane) for one species: 64 VGPRs either way, C4x10
  // 47-48 against 49-52 us (profiles/r06u_*); several species: single rows (three species with pairs: 98 VGPRs, 4 waves
  // per SIMD, C3 39.5 against 37.2 us).  PROM_TW_RP (read once): 1 or 2 forces either
  static const int rp_env = [] { const char* e = std::getenv("PROM_TW_RP"); return e ? std::atoi(e) : 0; }();
  const int rp = rp_env == 1 || rp_env == 2 ? rp_env : (nsig == 1 ? 2 : 1);
#define PROM_TWK(NS, DG, MGV)                                                                                        \
  if (rp == 2)                                                                                                       \
    hipExtLaunchKernelGGL((k_sigma_tw<NS, DG, MGV, 2>), dim3(nbw), dim3(kBlock), 0, s, ev0, ev1, 0, tabv, tabp, pc, wav, \
                          n_wav, n_rows, twseg, twrow, twlam, tr.n_tw, ta, ta.hdr, tabv.t[0].shift, ta.tab, ta.R);   \
  else                                                                                                               \
    hipExtLaunchKernelGGL((k_sigma_tw<NS, DG, MGV, 1>), dim3(nbw), dim3(kBlock), 0, s, ev0, ev1, 0, tabv, tabp, pc, wav, \
                          n_wav, n_rows, twseg, twrow, twlam, tr.n_tw, ta, ta.hdr, tabv.t[0].shift, ta.tab, ta.R)
#define PROM_TWD(NS, MGV)                 \
  if (deg <= 8) { PROM_TWK(NS, 8, MGV); } \
  else { PROM_TWK(NS, 14, MGV); }
  switch (nsig) {
    case 1: PROM_TWD(1, false) break;
    case 2: PROM_TWD(2, true) break;
    case 3: PROM_TWD(3, true) break;
    default: PROM_TWD(4, true) break;
  }
#undef PROM_TWD
#undef PROM_TWK
  PROM_HIP(hipGetLastError());
}

}  // namespace prom
