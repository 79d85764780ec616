// Doppler-shifted cross-section rows for the fast transit path (launched by launch_transit in
// prom_transit.hip when every phase has its own Doppler factor).
#include "prom_device.h"

namespace prom {

static_assert(kSigBlockW == kBlock, "sigma segments are built per kBlock wavelengths");
#ifndef PROM_SIG_FB_ROWS
#define PROM_SIG_FB_ROWS 1
#endif
constexpr int kSigFbRows = PROM_SIG_FB_ROWS;   // rows per gathering workgroup (independent lookups in flight per lane)
// minimum waves per SIMD the register allocation must allow (0: the compiler's choice, 70 VGPRs = 7 waves)
#ifndef PROM_SIG_WPE
#define PROM_SIG_WPE 0
#endif
#if PROM_SIG_WPE > 0
#define PROM_SIG_ATTR __attribute__((amdgpu_waves_per_eu(PROM_SIG_WPE)))
#else
#define PROM_SIG_ATTR
#endif

// ---- Doppler-shifted cross-section rows (orbital Doppler shift: one row per phase) ----------------
// The host (prom_api.hip sigma segments) gives, per 256-wavelength block and atomic slot, the table nodes
// [lo, lo + m) that every row's shifted targets shift_o * lambda_w fall between: positive factors and
// IEEE multiplication are monotone, so fl(shift_o lambda_w) lies in [fl(s_min lambda_first),
// fl(s_max lambda_last)].  Same bracket rule, slope, products and exp10 as sigma_of / sigma_multi: the
// rows are bit-for-bit those of the per-target lookups.

// One row's outputs at one wavelength: the cross sections (or the merged absorber Y and its zero flag).
// Returns the lane's Q value for the row's half-tile Q range, -1 when it is not finite or above 1e100.
template <int NSIG>
__device__ __forceinline__ float sigma_row_store(int32_t orow, int32_t nse, const double (&v)[NSIG],
                                                 const SigTabs4& tabv, bool live, int64_t w, int64_t n_wav,
                                                 int32_t merge_sp, double nscale_m, double* __restrict__ sig,
                                                 uint8_t* __restrict__ zfl) {
  double Qv = 0.0;
  if (merge_sp) {
    double Y = 0.0;
    bool z = false;
#pragma unroll
    for (int s = 0; s < NSIG; ++s) {
      const double cv = tabv.t[s].chi * v[s];
      if (!(cv > 0.0)) z = true;
      Y += cv;
    }
    if (live) {
      sig[(int64_t)orow * n_wav + w] = Y;
      zfl[(int64_t)orow * n_wav + w] = z ? 1u : 0u;
    }
    const double qs = Y * nscale_m;
    Qv = qs > 0.0 ? qs : 0.0;
  } else {
#pragma unroll
    for (int s = 0; s < NSIG; ++s) {
      if (live) sig[((int64_t)orow * nse + s) * n_wav + w] = v[s];
      const double qs = v[s] * tabv.t[s].nscale;
      Qv += qs > 0.0 ? qs : 0.0;
    }
  }
  return Qv <= 1.0e100 ? (float)Qv : -1.0f;
}

// A half tile's Q range from its lanes' values q (>= 0, or -1 for a non-finite one): [min q (1 - 2^-20),
// max q (1 + 2^-20)], or (-1, 0) when any value is -1.  (fl(q c) is monotone in q, so scaling after the
// min / max is the same as scaling every lane's value first.)
__device__ __forceinline__ float2 q_range(float qmin, float qmax) {
  return qmin < 0.0f ? make_float2(-1.0f, 0.0f) : make_float2(qmin * (1.0f - 0x1p-20f), qmax * (1.0f + 0x1p-20f));
}

// One row's outputs and its wavefront's half-tile Q range (DPP reductions over the 64 lanes).
template <int NSIG>
__device__ __forceinline__ void sigma_row_out(int32_t orow, int32_t nse, const double (&v)[NSIG], const SigTabs4& tabv,
                                              bool live, int64_t w, int64_t n_wav, int64_t hw, int64_t n_halves,
                                              int lane, int32_t merge_sp, double nscale_m, double* __restrict__ sig,
                                              float4* __restrict__ tq, uint8_t* __restrict__ zfl) {
  const float q = sigma_row_store<NSIG>(orow, nse, v, tabv, live, w, n_wav, merge_sp, nscale_m, sig, zfl);
  const float qh = wave_reduce_f(q, [](float a, float b) { return fmaxf(a, b); });
  const float ql = wave_reduce_f(q, [](float a, float b) { return fminf(a, b); });
  if (lane == 0 && hw < n_halves) reinterpret_cast<float2*>(tq)[(int64_t)orow * n_halves + hw] = q_range(ql, qh);
}

// Workgroups [0, n_blk * n_rc): one per (256-wavelength block whose slices all fit in LDS, chunk of
// kSigRowChunk rows).  Per species the block's node records go to LDS; a target's bracket comes from the
// slice's verified linear guess (interp_guess), so the rows' lookups are independent and their LDS round
// trips overlap.
// Workgroups [n_blk * n_rc, + n_fb * ceil(n_rows / kSigFbRows)): one per (other block, chunk of
// kSigFbRows rows) -- a species of these blocks has
// a slice larger than kSigSeg nodes (the high-resolution line windows, where the refined table is 10x
// finer than the grid and the rows' shifts spread the targets over thousands of nodes: the guess then
// reads the global records) or no verified guess (slices straddling a change of node spacing, targets
// outside the table: sigma_of's directory lookup).
template <int NSIG>
__global__ void __launch_bounds__(kBlock) PROM_SIG_ATTR k_sigma_rows(const SigTabs4 tabv, const double* __restrict__ wav, int64_t n_wav,
                                                 int32_t n_rows, const SigSeg* __restrict__ seg,
                                                 const int32_t* __restrict__ fb, int32_t n_fb, int32_t n_blk, int32_t n_rc,
                                                 double* __restrict__ sig, float4* __restrict__ tq, int32_t merge_sp,
                                                 double nscale_m, uint8_t* __restrict__ zfl) {
  // the slice as three conflict-free arrays: x (bracket tests), (x, f) pairs and slopes (the value)
  __shared__ double sx[kSigSeg];
  __shared__ double2 sxf[kSigSeg];
  __shared__ double ssl[kSigSeg];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int64_t n_halves = 2 * ((n_wav + kTW - 1) / kTW);
  const int32_t nse = merge_sp ? 1 : NSIG;
  const int64_t n_main = (int64_t)((n_blk + 7) / 8) * 8 * n_rc;
  if ((int64_t)blockIdx.x >= n_main) {
    // XCD-aware order as below: the row chunks of an oversize block are 8 workgroups apart, so its (large)
    // slice is fetched into one XCD's L2 rather than all eight
    const int64_t item = (int64_t)blockIdx.x - n_main;
    const int32_t n_fc = (n_rows + kSigFbRows - 1) / kSigFbRows;
    const int64_t fgrp = item / (8 * n_fc), frem = item % (8 * n_fc);
    const int64_t fi = fgrp * 8 + frem % 8;
    if (fi >= n_fb) return;
    const int32_t f0 = (int32_t)(frem / 8) * kSigFbRows;
    const int64_t wb = fb[fi];
    const int64_t w = wb * kBlock + tid;
    const bool live = w < n_wav;
    const double lam = wav[live ? w : n_wav - 1];
    double v[kSigFbRows][NSIG];
#pragma unroll
    for (int s = 0; s < NSIG; ++s) {
      const SigTabDev& tb = tabv.t[s];
      const SigSeg sg = seg[wb * NSIG + s];
      const double* __restrict__ gx = tb.x + sg.lo;
      const double* __restrict__ gy = tb.y + sg.lo;
#pragma unroll
      for (int r = 0; r < kSigFbRows; ++r) {
        const int32_t orow = f0 + r < n_rows ? f0 + r : n_rows - 1;
        const double t = tb.shift[orow] * lam;
        if ((sg.kind & 3) > 0) {
          // the x and f arrays (16 bytes per lane and array: the high-resolution slices are sparse in the
          // targets, so bytes per lane decide), the slope divided here as numpy does
          const int32_t g = seg_guess(t, sg.xs, sg.inv, sg.m);
          v[r][s] = exp10(interp_guess(
                        t, g, [&](int32_t i) { return make_double2(gx[i], gx[i + 1]); },
                        [&](int32_t i, double& x, double& f, double& sl) {
                          x = gx[i]; f = gy[i];
                          sl = (gy[i + 1] - f) / (gx[i + 1] - x);
                        })) - tb.offset;
        } else {
          v[r][s] = sigma_of(t, tb);
        }
      }
    }
    const int64_t hw = wb * (kBlock / 64) + (tid >> 6);
#pragma unroll
    for (int r = 0; r < kSigFbRows; ++r) {
      if (f0 + r >= n_rows) break;
      sigma_row_out<NSIG>(f0 + r, nse, v[r], tabv, live, w, n_wav, hw, n_halves, lane, merge_sp, nscale_m, sig, tq, zfl);
    }
    return;
  }
  // XCD-aware order (workgroup i runs on XCD i % 8): the n_rc row chunks of a block are 8 workgroups apart,
  // so they share an XCD's L2 for the block's slices
  const int64_t grp = blockIdx.x / (8 * n_rc), rem = blockIdx.x % (8 * n_rc);
  const int64_t wb = grp * 8 + rem % 8;
  const int32_t r0 = (int32_t)(rem / 8) * kSigRowChunk;
  if (wb >= n_blk) return;
  bool lds_ok = true;
#pragma unroll
  for (int s = 0; s < NSIG; ++s) lds_ok = lds_ok && (seg[wb * NSIG + s].kind & 3) == 1;
  if (!lds_ok) return;   // its rows are the trailing workgroups'
  const int64_t w = wb * kBlock + tid;
  const bool live = w < n_wav;
  const double lam = wav[live ? w : n_wav - 1];
  double V[kSigRowChunk][NSIG];
#pragma unroll
  for (int s = 0; s < NSIG; ++s) {
    const SigTabDev& tb = tabv.t[s];
    const SigSeg sg = seg[wb * NSIG + s];
    if (s > 0) __syncthreads();   // the previous species' slice is no longer read
    // the x and f arrays (16 bytes a node); slopes divided here, once per node and workgroup
    for (int32_t i = tid; i < sg.m; i += kBlock) {
      const double xv = tb.x[sg.lo + i], yv = tb.y[sg.lo + i];
      sx[i] = xv;
      sxf[i] = make_double2(xv, yv);
      if (i + 1 < sg.m) ssl[i] = (tb.y[sg.lo + i + 1] - yv) / (tb.x[sg.lo + i + 1] - xv);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSigRowChunk; ++r) {
      const int32_t orow = r0 + r < n_rows ? r0 + r : n_rows - 1;
      const double t = tb.shift[orow] * lam;
      const int32_t g = seg_guess(t, sg.xs, sg.inv, sg.m);
      V[r][s] = exp10(interp_guess(
                    t, g, [&](int32_t i) { return make_double2(sx[i], sx[i + 1]); },
                    [&](int32_t i, double& x, double& f, double& sl) {
                      const double2 q = sxf[i];
                      x = q.x; f = q.y; sl = ssl[i];
                    })) - tb.offset;
    }
  }
  // rows' outputs; their Q values go through LDS (over the slice, no longer read) so that the half-tile
  // ranges of all rows take one pass: thread (r, h, p) reduces 8 values, then 8 lanes combine by DPP
  constexpr bool kSqAlias = sizeof(double2) * kSigSeg >= sizeof(float) * kSigRowChunk * kBlock;
  __shared__ float sqx[kSqAlias ? 1 : kSigRowChunk * kBlock];
  float* sq = kSqAlias ? reinterpret_cast<float*>(sxf) : sqx;   // [kSigRowChunk][kBlock]
  float qv[kSigRowChunk];
#pragma unroll
  for (int r = 0; r < kSigRowChunk; ++r) {
    const int32_t orow = r0 + r < n_rows ? r0 + r : n_rows - 1;
    qv[r] = sigma_row_store<NSIG>(orow, nse, V[r], tabv, live && r0 + r < n_rows, w, n_wav, merge_sp, nscale_m,
                                  sig, zfl);
  }
  __syncthreads();   // every lane's lookups done: the slice arrays are free
#pragma unroll
  for (int r = 0; r < kSigRowChunk; ++r) sq[r * kBlock + tid] = qv[r];
  __syncthreads();
  {
    // TPH threads per (row, half tile), VPT values each, then log2(TPH) DPP steps
    constexpr int TPH = kBlock / (kSigRowChunk * 4), VPT = 64 / TPH;
    static_assert(TPH >= 4 && TPH <= 16 && TPH * VPT == 64, "4 to 16 threads per (row, half tile)");
    const int r = tid / (4 * TPH), h = (tid / TPH) & 3, pp = tid % TPH;
    const float* q8 = sq + r * kBlock + h * 64 + pp * VPT;
    float mn = q8[0], mx = q8[0];
#pragma unroll
    for (int i = 1; i < VPT; ++i) { mn = fminf(mn, q8[i]); mx = fmaxf(mx, q8[i]); }
    mn = fminf(mn, dpp_movf<0xB1>(mn)); mx = fmaxf(mx, dpp_movf<0xB1>(mx));     // quad_perm [1,0,3,2]
    mn = fminf(mn, dpp_movf<0x4E>(mn)); mx = fmaxf(mx, dpp_movf<0x4E>(mx));     // quad_perm [2,3,0,1]
    if (TPH >= 8) { mn = fminf(mn, dpp_movf<0x141>(mn)); mx = fmaxf(mx, dpp_movf<0x141>(mx)); }   // row_half_mirror
    if (TPH >= 16) { mn = fminf(mn, dpp_movf<0x140>(mn)); mx = fmaxf(mx, dpp_movf<0x140>(mx)); }  // row_mirror
    const int64_t hw2 = wb * (kBlock / 64) + h;
    if (pp == 0 && r0 + r < n_rows && hw2 < n_halves)
      reinterpret_cast<float2*>(tq)[(int64_t)(r0 + r) * n_halves + hw2] = q_range(mn, mx);
  }
}

// ---- polynomial sigma rows (prom_transit_set: sig_deg > 0) ---------------------------------------------
// On numpy's bracket [x_k, x_{k+1}) of a target t,
//   sigma_s(t) = 10^(f_k + slope_k (t - x_k)) - offset = E_k e^a - offset,   a = L_k (t - x_k),
// with E_k = 10^f_k and L_k = ln10 slope_k kept per node (AtomTable::rec, k_table_recs).  e^a is a degree-D
// Taylor polynomial: the tables bound |a| on every interval by amax (AtomTable::amax) and prom_transit_set
// takes the smallest even D with e^amax amax^(D+1)/(D+1)! <= 2^-53, so the truncation is below one rounding of
// e^a.
// (The remainder relative to e^a carries e^|a| when a < 0: prom_transit_set's rule includes that factor.)
// Against numpy's 10^v (v rounded once) sigma moves by ~|v| ln10 2^-53 (about 1e-14 relative); at an exact
// node hit a = 0 and sigma is 10^f_k - offset as numpy's node rule gives it, and a flat interval at the
// table floor (10^-50) gives exactly 0, so the exact path's zero pattern is kept.  No exp10, no division:
// about 10 + D FP64 operations per lookup against ~33 on the exp10 path.
// (InvFact, PolyCoef, exp_taylor: prom_device.h, shared with the fused tau kernel)

#ifndef PROM_SIG_POLY_ROWS
#define PROM_SIG_POLY_ROWS 0
#endif
constexpr int kSigPolyRows = PROM_SIG_POLY_ROWS;   // rows (phases) per workgroup of k_sigma_poly (4 or 8; 0: per problem)

// One workgroup per (256-wavelength block, chunk of R rows).  Blocks whose slices all fit in LDS: per species
// the block's records {x_k, x_{k+1}} and {E_k, L_k} go to LDS; kind & 4 (the guess is numpy's bracket for
// every target, k_seg_exact): one LDS round trip per lookup, else the +-1 bracket test and a second one.
// The rows accumulate Y (merged species) or store sigma_s and their Q sum, species after species.  Oversize
// blocks (fb, dispatched first): records read from the global table (one 32-byte record, a second only for
// lanes whose bracket is the guess +- 1), or sigma_poly_of without a guess.  (The row path: several unmerged
// species with orbital Doppler shift, or PROM_TCURVE=0; one effective absorber takes k_sigma_tc.)
template <int NSIG, int D, bool MG, int R>
__global__ void __launch_bounds__(kBlock) PROM_SIG_ATTR k_sigma_poly(const SigTabs4 tabv, const PolyCoef pc,
                                                       const double* __restrict__ wav, int64_t n_wav,
                                                       int32_t n_rows, const SigSeg* __restrict__ seg,
                                                       const int32_t* __restrict__ fb, int32_t n_fb, int32_t n_blk,
                                                       int32_t n_rc, double* __restrict__ sig, float4* __restrict__ tq,
                                                       int32_t merge_sp, double nscale_m, uint8_t* __restrict__ zfl,
                                                       int32_t rf) {
  static_assert(R == 4 || R == 8, "4 or 8 rows per workgroup");
  // per staged species: [0, kSigSeg) {x_k, x_{k+1}}, [kSigSeg, 2 kSigSeg) {E_k, L_k}
  __shared__ double2 slds[2 * kSigSeg];
  double2* sxr = slds;
  double2* sel = slds + kSigSeg;
  const int tid = threadIdx.x;
  const int64_t n_halves = 2 * ((n_wav + kTW - 1) / kTW);
  const int32_t nse = MG ? 1 : NSIG;
  // one workgroup per (256-wavelength block, chunk of R rows), XCD-aware: the row chunks of a block are 8
  // workgroups apart (one XCD's L2 for its slices).  The oversize blocks (fb, global-record lookups: a chain of
  // L2 / HBM round trips per workgroup, the long pole) come first, their row chunks n_fb8 workgroups apart;
  // front workgroups take rf <= R rows (more of them in flight).  The LDS blocks follow.
  const int32_t RF = rf;
  const int64_t n_fb8 = ((int64_t)n_fb + 7) / 8 * 8, n_front = n_fb8 * ((n_rows + RF - 1) / RF);
  int64_t bid = blockIdx.x, wb;
  int32_t r0, rcap = R;   // rows [r0, min(r0 + rcap, n_rows)) are this workgroup's
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
#pragma unroll
    for (int s = 0; s < NSIG; ++s) lds_ok = lds_ok && (seg[wb * NSIG + s].kind & 3) == 1;
    if (!lds_ok) return;   // (a front workgroup's)
  }
  const int32_t rlim = r0 + rcap < n_rows ? r0 + rcap : n_rows;
  rcap = rlim - r0;   // rows present (front workgroups: no lookups for padding rows)
#ifdef PROM_TRACE
  const unsigned long long tr_t0 = wall_clock64();
#endif
  const int64_t w = wb * kBlock + tid;
  const bool live = w < n_wav;
  const double lam = wav[live ? w : n_wav - 1];
  double acc[R];        // merged: Y = sum_s chi_s sigma_s;  else: Q = sum_s max(sigma_s / c_s, 0)
  uint32_t zb = 0;      // merged: bit r set when some chi_s sigma_s is not > 0
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0;
#pragma unroll
  for (int s = 0; s < NSIG; ++s) {
    const SigTabDev& tb = tabv.t[s];
    const SigSeg sg = seg[wb * NSIG + s];
    if (lds_ok) {
      if (s > 0) __syncthreads();   // the previous species' slice is no longer read
      for (int32_t i = tid; i < sg.m; i += kBlock) {
        const double4 q = tb.rec[sg.lo + i];
        sxr[i] = make_double2(q.x, q.w);
        sel[i] = make_double2(q.y, q.z);
      }
      __syncthreads();
    }
    const bool exact = (sg.kind & 4) != 0;
    const double off = tb.offset, chi = tb.chi, nsc = tb.nscale;
    auto emit = [&](int r, double v) {
      const int32_t orow = r0 + r;
      if constexpr (MG) {
        const double cv = chi * v;
        if (!(cv > 0.0)) zb |= 1u << r;
        acc[r] += cv;
      } else {
        if (sig && live && orow < rlim) sig[((int64_t)orow * nse + s) * n_wav + w] = v;
        const double qs = v * nsc;
        acc[r] += qs > 0.0 ? qs : 0.0;
      }
    };
    // the rows' targets first (scalar loads of the Doppler factors, one wait), so that the lookups' LDS reads
    // are not serialised behind them (lgkmcnt counts scalar loads and LDS reads together)
    double tt[R];
#pragma unroll
    for (int r = 0; r < R; ++r) tt[r] = tb.shift[r0 + r < n_rows ? r0 + r : n_rows - 1] * lam;
    if (!lds_ok) {
      if ((sg.kind & 3) > 0) {
        // groups of G rows: G records in flight per lane
        constexpr int G = 4;
        const double4* __restrict__ rr = tb.rec + sg.lo;
#pragma unroll
        for (int r0g = 0; r0g < R; r0g += G) {
          if (r0g >= rcap) break;
          double4 q[G];
#pragma unroll
          for (int j = 0; j < G; ++j) q[j] = rr[seg_guess(tt[r0g + j], sg.xs, sg.inv, sg.m)];
          if (!exact) {
#pragma unroll
            for (int j = 0; j < G; ++j) {
              const double t = tt[r0g + j];
              const int32_t g = seg_guess(t, sg.xs, sg.inv, sg.m);
              const int32_t k = t < q[j].x ? g - 1 : (t >= q[j].w ? g + 1 : g);
              if (k != g) q[j] = rr[k];
            }
          }
#pragma unroll
          for (int j = 0; j < G; ++j)
            emit(r0g + j, __builtin_fma(q[j].y, exp_taylor<D>(q[j].z * (tt[r0g + j] - q[j].x), pc), -off));
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (r < rcap) emit(r, sigma_poly_of(tt[r], tb, pc, D));
      }
    } else {
      // rows past rcap (a problem with fewer rows than R) are skipped; the guarded copy only runs then (the
      // unguarded one keeps the rows' LDS reads free to overlap)
      auto lds_rows = [&](auto guard) {
        constexpr bool GD = decltype(guard)::value;
        double xk[R];
        double2 el[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (GD && r >= rcap) break;
          const int32_t g = seg_guess(tt[r], sg.xs, sg.inv, sg.m);
          if (exact) {
            xk[r] = sxr[g].x;
            el[r] = sel[g];
          } else {
            const double2 xx = sxr[g];
            const int32_t k = tt[r] < xx.x ? g - 1 : (tt[r] >= xx.y ? g + 1 : g);
            xk[r] = sxr[k].x;
            el[r] = sel[k];
          }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (GD && r >= rcap) break;
          emit(r, __builtin_fma(el[r].x, exp_taylor<D>(el[r].y * (tt[r] - xk[r]), pc), -off));
        }
      };
      if (rcap >= R) lds_rows(std::false_type{});
      else lds_rows(std::true_type{});
    }
  }
  // rows' outputs, then their half-tile Q ranges through LDS (over the slices, no longer read)
  float qv[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int32_t orow = r0 + r;
    double Qv;
    if constexpr (MG) {
      if (sig && live && orow < rlim) {
        sig[(int64_t)orow * n_wav + w] = acc[r];
        zfl[(int64_t)orow * n_wav + w] = (zb >> r) & 1u;
      }
      const double qs = acc[r] * nscale_m;
      Qv = qs > 0.0 ? qs : 0.0;
    } else {
      Qv = acc[r];
    }
    qv[r] = Qv <= 1.0e100 ? (float)Qv : -1.0f;
  }
  static_assert(sizeof(double2) * 2 * kSigSeg >= sizeof(float) * R * kBlock, "Q staging fits over the slices");
  float* sq = reinterpret_cast<float*>(slds);   // [R][kBlock]
  __syncthreads();   // every lane's lookups done: the slices are free
#pragma unroll
  for (int r = 0; r < R; ++r) sq[r * kBlock + tid] = qv[r];
  __syncthreads();
  {
    constexpr int TPH = kBlock / (R * 4), VPT = 64 / TPH;
    static_assert(TPH >= 4 && TPH <= 16 && TPH * VPT == 64, "4 to 16 threads per (row, half tile)");
    const int r = tid / (4 * TPH), h = (tid / TPH) & 3, pp = tid % TPH;
    const float* q8 = sq + r * kBlock + h * 64 + pp * VPT;
    float mn = q8[0], mx = q8[0];
#pragma unroll
    for (int i = 1; i < VPT; ++i) { mn = fminf(mn, q8[i]); mx = fmaxf(mx, q8[i]); }
    mn = fminf(mn, dpp_movf<0xB1>(mn)); mx = fmaxf(mx, dpp_movf<0xB1>(mx));     // quad_perm [1,0,3,2]
    mn = fminf(mn, dpp_movf<0x4E>(mn)); mx = fmaxf(mx, dpp_movf<0x4E>(mx));     // quad_perm [2,3,0,1]
    if (TPH >= 8) { mn = fminf(mn, dpp_movf<0x141>(mn)); mx = fmaxf(mx, dpp_movf<0x141>(mx)); }   // row_half_mirror
    if (TPH >= 16) { mn = fminf(mn, dpp_movf<0x140>(mn)); mx = fmaxf(mx, dpp_movf<0x140>(mx)); }  // row_mirror
    const int64_t hw2 = wb * (kBlock / 64) + h;
    if (pp == 0 && r0 + r < rlim && hw2 < n_halves)
      reinterpret_cast<float2*>(tq)[(int64_t)(r0 + r) * n_halves + hw2] = q_range(mn, mx);
  }
#ifdef PROM_TRACE
  // per workgroup: start, end (wall clock, 10 ns), block | lds << 32 | front << 33, first row | HW_ID << 32
  if (threadIdx.x == 0 && blockIdx.x < (1u << 18)) {
    unsigned long long* tp = g_trace + 4ull * blockIdx.x;
    tp[0] = tr_t0;
    tp[1] = wall_clock64();
    tp[2] = (unsigned long long)wb | ((unsigned long long)lds_ok << 32) | ((unsigned long long)(blockIdx.x < n_front) << 33);
    unsigned long long kinds = 0;   // 3 bits per species, then the largest slice
    int32_t mmax = 0;
    for (int s = 0; s < NSIG; ++s) {
      kinds |= (unsigned long long)(seg[wb * NSIG + s].kind & 7) << (3 * s);
      mmax = seg[wb * NSIG + s].m > mmax ? seg[wb * NSIG + s].m : mmax;
    }
    tp[3] = (unsigned long long)(uint32_t)r0 | (kinds << 32) | ((unsigned long long)(mmax > 65535 ? 65535 : mmax) << 44);
  }
#endif
}

#ifdef PROM_TRACE
extern "C" int32_t prom_sig_trace_read(unsigned long long* out, int32_t n, int32_t clear) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_trace), sizeof(unsigned long long) * n) != hipSuccess) return -1;
  if (clear) {
    static unsigned long long zeros[1 << 20];
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_trace), zeros, sizeof(zeros)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// prom_transit_set: flags[b][s] = 1 when the guess of segment (b, s) differs from numpy's bracket for some
// target shift_o lambda_w of the block (every row, and the last wavelength for lanes past n_wav, as the
// sigma-row kernels take it); k_seg_mark then sets kind |= 4 on the others.
template <int NSIG>
__global__ void __launch_bounds__(kBlock) k_seg_exact(const SigTabs4 tabv, const double* __restrict__ wav, int64_t n_wav,
                                                      int32_t n_rows, const SigSeg* __restrict__ seg,
                                                      int32_t* __restrict__ flags) {
  const int64_t wb = blockIdx.x;
  const int64_t w = wb * kBlock + threadIdx.x;
  const double lam = wav[w < n_wav ? w : n_wav - 1];
#pragma unroll
  for (int s = 0; s < NSIG; ++s) {
    const SigSeg sg = seg[wb * NSIG + s];
    if ((sg.kind & 3) == 0) continue;
    const SigTabDev& tb = tabv.t[s];
    const double* __restrict__ X = tb.x + sg.lo;
    bool ok = true;
    for (int32_t o = 0; o < n_rows; ++o) {
      const double t = tb.shift[o] * lam;
      const int32_t g = seg_guess(t, sg.xs, sg.inv, sg.m);
      int32_t a = 0, b = sg.m - 1;   // X[a] <= t < X[b] (the host's slice bounds)
      while (b - a > 1) {
        const int32_t mid = (a + b) >> 1;
        if (X[mid] <= t) a = mid; else b = mid;
      }
      ok = ok && a == g;
    }
    if (__ballot(!ok) != 0ull && (threadIdx.x & 63) == 0) atomicOr(&flags[wb * NSIG + s], 1);
  }
}

__global__ void k_seg_mark(SigSeg* __restrict__ seg, const int32_t* __restrict__ flags, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  if (i < n && (seg[i].kind & 3) != 0 && flags[i] == 0) seg[i].kind |= 4;
}

void launch_seg_exact(hipStream_t s, int32_t nsig, const SigTabs4& tabv, const double* wav, int64_t n_wav,
                      int32_t n_rows, SigSeg* seg, int32_t* flags) {
  const int64_t n_blk = (n_wav + kBlock - 1) / kBlock;
  PROM_HIP(hipMemsetAsync(flags, 0, sizeof(int32_t) * n_blk * nsig, s));
#define PROM_SE(NS) \
  hipLaunchKernelGGL((k_seg_exact<NS>), dim3((unsigned)n_blk), dim3(kBlock), 0, s, tabv, wav, n_wav, n_rows, seg, flags)
  switch (nsig) {
    case 1: PROM_SE(1); break;
    case 2: PROM_SE(2); break;
    case 3: PROM_SE(3); break;
    default: PROM_SE(4); break;
  }
#undef PROM_SE
  PROM_HIP(hipGetLastError());
  hipLaunchKernelGGL(k_seg_mark, dim3(grid_for(n_blk * nsig)), dim3(kBlock), 0, s, seg, flags, n_blk * nsig);
  PROM_HIP(hipGetLastError());
}

void launch_sigma_poly(hipStream_t s, int32_t nsig, int32_t deg, const SigTabs4& tabv, const double* wav, int64_t n_wav,
                       int32_t n_rows, const SigSeg* seg, const int32_t* fb, int32_t n_fb, double* sig, float4* tq,
                       int32_t merge_sp, double nscale_m, uint8_t* zfl, hipEvent_t ev_start, hipEvent_t ev_stop) {
  const int32_t n_blk = (int32_t)grid_for(n_wav);
  // rows per workgroup: PROM_SIG_POLY_ROWS when set at build time, else 8 for several species (their lookups
  // fill the workgroup) and 4 for one (more workgroups in flight)
  const int R = kSigPolyRows > 0 ? kSigPolyRows : (nsig >= 2 ? 8 : 4);
  const int32_t n_rc = (n_rows + R - 1) / R;
  // rows per front workgroup (measured, profiles/r03_sigma_rf_sweep.txt): R / 2 for several species (C3: 4
  // of 8 rows, 37 against 49 us isolated); one species: all R rows when there are >= 16384 (block, row)
  // pairs of oversize blocks, else R / 2
  const int RF = (nsig >= 2 || (int64_t)n_fb * n_rows < 16384) ? R / 2 : R;
  const int64_t n_front = (int64_t)((n_fb + 7) / 8) * 8 * ((n_rows + RF - 1) / RF);
  const unsigned nb = (unsigned)(n_front + (n_fb >= n_blk ? 0 : (int64_t)((n_blk + 7) / 8) * 8 * n_rc));
  const PolyCoef& pc = poly_coef();
#define PROM_SIGK(NS, DG, MGV, RV)                                                                             \
  hipExtLaunchKernelGGL((k_sigma_poly<NS, DG, MGV, RV>), dim3(nb), dim3(kBlock), 0, s, ev_start, ev_stop, 0,   \
                        tabv, pc, wav, n_wav, n_rows, seg, fb, n_fb, n_blk, n_rc, sig, tq, merge_sp, nscale_m, zfl, RF)
#define PROM_SIGP(NS, DG, MGT)                                                   \
  do {                                                                           \
    if (merge_sp && R == 8) PROM_SIGK(NS, DG, true, 8);                          \
    else if (merge_sp) PROM_SIGK(NS, DG, true, 4);                               \
    else if (R == 8) PROM_SIGK(NS, DG, false, 8);                                \
    else PROM_SIGK(NS, DG, false, 4);                                            \
  } while (0)
  // degree 8 covers every table with amax <= 0.07 (the high-resolution configs), 14 the rest
#define PROM_SIGP_D(NS, MGT)                 \
  if (deg <= 8) PROM_SIGP(NS, 8, MGT);       \
  else PROM_SIGP(NS, 14, MGT);
  switch (nsig) {
    case 1: PROM_SIGP_D(1, false) break;
    case 2: PROM_SIGP_D(2, true) break;
    case 3: PROM_SIGP_D(3, true) break;
    default: PROM_SIGP_D(4, true) break;
  }
#undef PROM_SIGP_D
#undef PROM_SIGP
#undef PROM_SIGK
  PROM_HIP(hipGetLastError());
}

void launch_sigma_rows(hipStream_t s, int32_t nsig, const SigTabs4& tabv, const double* wav, int64_t n_wav,
                       int32_t n_rows, const SigSeg* seg, const int32_t* fb, int32_t n_fb, double* sig, float4* tq,
                       int32_t merge_sp, double nscale_m, uint8_t* zfl, hipEvent_t ev_start, hipEvent_t ev_stop) {
  const int32_t n_blk = (int32_t)grid_for(n_wav);
  const int32_t n_rc = (n_rows + kSigRowChunk - 1) / kSigRowChunk;
  const int32_t n_fc = (n_rows + kSigFbRows - 1) / kSigFbRows;
  const unsigned nb = (unsigned)((int64_t)((n_blk + 7) / 8) * 8 * n_rc + (int64_t)((n_fb + 7) / 8) * 8 * n_fc);
#define PROM_SIGR(NS)                                                                                        \
  hipExtLaunchKernelGGL((k_sigma_rows<NS>), dim3(nb), dim3(kBlock), 0, s, ev_start, ev_stop, 0, tabv, wav, n_wav, \
                        n_rows, seg, fb, n_fb, n_blk, n_rc, sig, tq, merge_sp, nscale_m, zfl)
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
