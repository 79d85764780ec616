// k_sigma_tw: the Doppler-shifted cross-section lookups and transmission curves over target windows.
// Compiled in its own translation unit with machine LICM off (build.py): hoisting the rare passes' constants (ocml exp
// coefficients, directory-search state) out of the item loop held ~30 VGPRs for the whole kernel (87 -> 54 VGPRs).
#include "prom_tc.h"

namespace prom {

// ---- sigma lookups + transmission curves over target windows (the default with orbital Doppler shift) ------
// The targets t = shift_o lambda_w of all rows, not the wavelengths, are cut into windows (host: prom_window.hip):
// window b holds, per row o, the contiguous wavelengths w in [W[b][o], W[b+1][o]) whose targets fall in the
// window's target interval (at most a few hundred per row).  Per species the table nodes those targets reach are
// one slice, staged once per window for every row: no Doppler-spread overlap between neighbouring windows' slices
// and no second workgroup staging the same slice for other rows.  All species share one pool of kTwPool nodes
// (24 bytes a node: 19 KB a workgroup).  Work items are (row, 64 wavelengths) with the row wave-uniform: its
// Doppler factor, curve header and coefficients are scalar loads.  Per species slice (SigSeg kind & 3): 1 staged,
// with the host-verified linear guess (one LDS round: x_g, x_{g+1} and the record; a second only for lanes one
// node off); 2 the same guess into the global records (a slice larger than the pool); 0 none (targets outside the
// table, or no guess): the window goes to the second pass.  The second pass also takes the rows whose curve header
// says non-finite columns (flag 2, the reference's chord order) or a table truncated at the host's octave cap
// (flag 4, the exact sum beyond it): numpy's bracket from the table's directory, per point.  Every path evaluates
// fl(chi E_k) e^a (or E_k e^a - offset) of numpy's bracket k, so R does not depend on the windows: bitwise equal
// to k_sigma_tc's and for any wavelength or phase shard.  Keeping the rare paths out of the first pass keeps its
// register peak low (no ocml exp, no directory search live beside the lookups).
constexpr int kTwPool = kTwPoolMax;

template <int NSIG, int D, bool MG>
__global__ void __launch_bounds__(kBlock) k_sigma_tw(const SigTabs4 tabv, const PolyCoef pc, const double* __restrict__ wav,
                                                     int64_t n_wav, int32_t n_rows, const SigSeg* __restrict__ wseg,
                                                     const int32_t* __restrict__ wrow, int32_t n_win, const TcArgs ta) {
  static_assert(D > 0, "polynomial lookups only (coarse tables take k_sigma_tc)");
  __shared__ double sx[kTwPool + 4];       // species s: x_lo .. x_{lo+m} at pad + s
  __shared__ double2 sel[kTwPool];         // species s: {(chi) E_k, L_k} at pad
  // XCD-aware: workgroup ids round-robin over the 8 XCDs; XCD x takes windows [x per, (x + 1) per) in order, so
  // neighbouring windows (whose rows read overlapping wavelengths) share an L2
  const int32_t per = (n_win + 7) >> 3;
  const int32_t b = (int32_t)(blockIdx.x & 7) * per + (int32_t)(blockIdx.x >> 3);
  if (b >= n_win) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  SigSeg sg[NSIG];
  bool wrare = false;   // (some species without a slice: second pass for the whole window)
#pragma unroll
  for (int s = 0; s < NSIG; ++s) {
    sg[s] = wseg[(int64_t)b * NSIG + s];
    wrare = wrare || (sg[s].kind & 3) == 0;
  }
  // stage the kind-1 slices: pool entry i belongs to the species whose [pad, pad + m) holds it; every load issued
  // before the first LDS write
  {
    constexpr int NQ = (kTwPool + kBlock - 1) / kBlock;
    int32_t tot = 0;
#pragma unroll
    for (int s = 0; s < NSIG; ++s)
      if ((sg[s].kind & 3) == 1) tot = sg[s].pad + sg[s].m > tot ? sg[s].pad + sg[s].m : tot;
    double4 q[NQ];
    int sp[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const int32_t i = tid + j * kBlock;
      sp[j] = -1;
#pragma unroll
      for (int s = 0; s < NSIG; ++s)
        if ((sg[s].kind & 3) == 1 && i >= sg[s].pad && i < sg[s].pad + sg[s].m) sp[j] = s;
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
  }
  __syncthreads();
  double choff = 0.0;
  if constexpr (MG) {
#pragma unroll
    for (int s = 0; s < NSIG; ++s) choff += tabv.t[s].chi * tabv.t[s].offset;
  }
  const int32_t* __restrict__ wa = wrow + (int64_t)b * n_rows;
  const int32_t* __restrict__ wz = wa + n_rows;
  // items (row o, chunk c of 64 wavelengths), item k of a pass to wave k mod 4, rows walked in order (scalar);
  // pass 0 takes the rows the first pass can do, pass 1 the others
  for (int pass = 0; pass < 2; ++pass) {
    int32_t o = 0, c = wv;
    while (true) {
      int32_t w0 = 0, w1 = 0;
      while (o < n_rows) {
        const bool rare = wrare || ((int32_t)ta.hdr[(int64_t)o * kTcHdr + kTcHFlags] & 6) != 0;
        if (rare == (pass == 1)) {
          w0 = wa[o];
          w1 = wz[o];
          const int32_t nch = (w1 - w0 + 63) >> 6;
          if (c < nch) break;
          c -= nch;
        }
        ++o;
      }
      if (o >= n_rows) break;
      const int32_t w = w0 + c * 64 + lane;
      const bool live = w < w1;
      const double lam = wav[live ? w : w1 - 1];
      const double t = tabv.t[0].shift[o] * lam;
      const double* h = ta.hdr + (int64_t)o * kTcHdr;
      double acc = 0.0, v;
      if (pass == 0) {
#pragma unroll
        for (int s = 0; s < NSIG; ++s) {
          const SigSeg& ss = sg[s];
          const int32_t g = seg_guess(t, ss.xs, ss.inv, ss.m);
          double ce, x0, sl;
          if ((ss.kind & 3) == 1) {
            const double* xs = sx + ss.pad + s;
            const double2* el = sel + ss.pad;
            x0 = xs[g];
            const double x1 = xs[g + 1];
            double2 e = el[g];
            if (t < x0 || t >= x1) {   // (rare: the guess is one node off)
              const int32_t k = t < x0 ? g - 1 : g + 1;
              x0 = xs[k];
              e = el[k];
            }
            ce = e.x;
            sl = e.y;
          } else {
            const double4* __restrict__ rr = tabv.t[s].rec + ss.lo;
            double4 q = rr[g];
            const int32_t k = t < q.x ? g - 1 : (t >= q.w ? g + 1 : g);
            if (k != g) q = rr[k];
            ce = MG ? tabv.t[s].chi * q.y : q.y;
            x0 = q.x;
            sl = q.z;
          }
          const double ex = exp_taylor<D>(sl * (t - x0), pc);
          if constexpr (MG) acc = __builtin_fma(ce, ex, acc);
          else acc = __builtin_fma(ce, ex, -tabv.t[s].offset);
        }
        if constexpr (MG) acc -= choff;
        v = tc_eval_full(acc, h, ta.tab + (int64_t)o * ta.lg * kTcD);
      } else {
        // second pass: numpy's bracket per point; zr (merged species, non-finite columns): some chi_s sigma_s not > 0
        bool zr = false;
#pragma unroll
        for (int s = 0; s < NSIG; ++s) {
          const SigTabDev& tb = tabv.t[s];
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
          v = tc_eval_full(Y, h, ta.tab + (int64_t)o * ta.lg * kTcD);
        } else {
          const int32_t* fl = ta.flags + (int64_t)o * ta.n_pr;
          const double* nc = ta.ncol + (int64_t)o * ta.n_pr;
          const double fs = h[kTcHFsum], inv_fs = 1.0 / fs;
          double a = 0.0;
#pragma unroll 1
          for (int32_t ci = 0; ci < ta.n_pr; ++ci) {
            if (fl[ci] != 0) continue;
            const double N = nc[ci];
            double tau = N * Y;
            if (nf && zr && !__builtin_isfinite(N)) tau = __builtin_nan("");
            const double e = exp(-tau);
            a = nf ? a + ta.fout[ci] * e : a + (ta.fout[ci] * inv_fs) * e;
          }
          if (beyond && ta.evals) atomicAdd(&ta.evals[threadIdx.x & 63], (unsigned long long)(int32_t)h[kTcHNact]);
          v = nf ? (a + h[kTcHTfrac] * fs) / fs : h[kTcHTfrac] + a;
        }
      }
      if (live) ta.R[(int64_t)o * n_wav + w] = v;
      c += 4;
    }
  }
}

void launch_sigma_tw(hipStream_t s, TransitDev& tr, int32_t nsig, int32_t deg, const TcArgs& ta, hipEvent_t ev0,
                     hipEvent_t ev1) {
  const unsigned nbw = (unsigned)(((int64_t)tr.n_tw + 7) / 8 * 8);   // one workgroup per window, XCD-interleaved ids
  const SigSeg* twseg = tr.tw_seg.as<SigSeg>();
  const int32_t* twrow = tr.tw_row.as<int32_t>();
  const PolyCoef& pc = poly_coef();
  const SigTabs4& tabv = tr.sigtab_v;
  const double* wav = tr.wav.as<double>();
  const int32_t n_rows = tr.n_orb;
  const int64_t n_wav = tr.n_wav;
  PROM_REQUIRE(deg > 0 && n_rows >= 2 && tr.n_tw > 0, "k_sigma_tw: polynomial lookups with orbital Doppler rows");
#define PROM_TWK(NS, DG, MGV)                                                                                  \
  hipExtLaunchKernelGGL((k_sigma_tw<NS, DG, MGV>), dim3(nbw), dim3(kBlock), 0, s, ev0, ev1, 0, tabv, pc, wav, n_wav, \
                        n_rows, twseg, twrow, tr.n_tw, ta)
#define PROM_TWD(NS, MGV)                 \
  if (deg <= 8) PROM_TWK(NS, 8, MGV);     \
  else PROM_TWK(NS, 14, MGV);
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
