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
// main workgroups' table access: 0 one species' slice in LDS at a time; 1 every species' slice staged at once;
// 2 no LDS, records read from the global table
#ifndef PROM_SIG_MODE
#define PROM_SIG_MODE 0
#endif
constexpr int kSigMode = PROM_SIG_MODE;
#ifndef PROM_SIG_NOSTORE
#define PROM_SIG_NOSTORE 0
#endif
constexpr bool kSigNoStore = PROM_SIG_NOSTORE != 0;   // profiling only: no sigma-row / zero-flag stores

// One workgroup per (256-wavelength block, chunk of R rows).  Blocks whose slices all fit in LDS: per species
// the block's records {x_k, x_{k+1}} and {E_k, L_k} go to LDS; kind & 4 (the guess is numpy's bracket for
// every target, k_seg_exact): one LDS round trip per lookup, else the +-1 bracket test and a second one.
// The rows accumulate Y (merged species) or their Q sum in registers, species after species.  Oversize
// blocks (fb, dispatched first): records read from the global table (one 32-byte record, a second only for
// lanes whose bracket is the guess +- 1), or sigma_poly_of without a guess.
// TAU (fused Doppler path, one effective absorber: merged species or one species): no rows are stored; after
// the Q ranges the workgroup integrates its (row, half tile) windows itself (k_windows' window choice and
// k_tau_p's static-unit arithmetic, so R is bit for bit that of the row path) and hands the heavy half tiles
// (window > kHeavy records) to k_tau_p as entries, storing Y for those half tiles only.
template <int NSIG, int D, bool MG, int R, bool TAU>
__global__ void __launch_bounds__(kBlock) PROM_SIG_ATTR k_sigma_poly(const SigTabs4 tabv, const PolyCoef pc,
                                                       const double* __restrict__ wav, int64_t n_wav,
                                                       int32_t n_rows, const SigSeg* __restrict__ seg,
                                                       const int32_t* __restrict__ fb, int32_t n_fb, int32_t n_blk,
                                                       int32_t n_rc, double* __restrict__ sig, float4* __restrict__ tq,
                                                       int32_t merge_sp, double nscale_m, uint8_t* __restrict__ zfl,
                                                       int32_t parts, int32_t rf, const TauArgs ta) {
  static_assert(R == 4 || R == 8 || R == 16, "4, 8 or 16 rows per workgroup");
  static_assert(!TAU || MG || NSIG == 1, "the fused integration takes one effective absorber");
  // per staged species: [0, kSigSeg) {x_k, x_{k+1}}, [kSigSeg, 2 kSigSeg) {E_k, L_k}
  __shared__ double2 slds[2 * kSigSeg * (kSigMode == 1 ? NSIG : 1)];
  double2* sxr = slds;
  double2* sel = slds + kSigSeg;
  const int tid = threadIdx.x;
  const int64_t n_halves = 2 * ((n_wav + kTW - 1) / kTW);
  const int32_t nse = MG ? 1 : NSIG;
  // one workgroup per (256-wavelength block, chunk of R rows), XCD-aware: the row chunks of a block are 8
  // workgroups apart (one XCD's L2 for its slices)
  // The oversize blocks (fb, global-record lookups: a chain of L2 / HBM round trips per workgroup, the long
  // pole) come first, so that they are not the last workgroups dispatched; their row chunks are n_fb8
  // workgroups apart (one XCD).  The LDS blocks follow, in the XCD-aware order; oversize ones exit there.
  // front workgroups take rf <= R rows (more of them in flight: their lookups are a chain of round trips)
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
  // PROM_SIG_PARTS (profiling only): 1 = LDS blocks, 2 = global-record blocks
  if (!(parts & (lds_ok ? 1 : 2))) return;
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
  double sv[(TAU && !MG) ? R : 1];   // TAU, one species: the row's sigma (acc holds its Q)
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0;
  constexpr int kPre = kSigSeg / kBlock;   // mode 3: records per thread and species (slices <= kSigSeg nodes)
  double4 pre[kPre];
  auto fetch = [&](int s) {
    const SigSeg sg = seg[wb * NSIG + s];
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const int32_t i = tid + j * kBlock;
      pre[j] = i < sg.m ? tabv.t[s].rec[sg.lo + i] : make_double4(0.0, 0.0, 0.0, 0.0);
    }
  };
  if (kSigMode == 3 && lds_ok) fetch(0);
  if (kSigMode == 1 && lds_ok) {
    // every species' slice staged at once (one global round trip; NSIG x 16 KB of LDS)
#pragma unroll
    for (int s = 0; s < NSIG; ++s) {
      const SigSeg sg = seg[wb * NSIG + s];
      for (int32_t i = tid; i < sg.m; i += kBlock) {
        const double4 q = tabv.t[s].rec[sg.lo + i];
        slds[s * 2 * kSigSeg + i] = make_double2(q.x, q.w);
        slds[s * 2 * kSigSeg + kSigSeg + i] = make_double2(q.y, q.z);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int s = 0; s < NSIG; ++s) {
    const SigTabDev& tb = tabv.t[s];
    const SigSeg sg = seg[wb * NSIG + s];
    const double2* __restrict__ sx_ = kSigMode == 1 ? slds + s * 2 * kSigSeg : sxr;
    const double2* __restrict__ se_ = kSigMode == 1 ? slds + s * 2 * kSigSeg + kSigSeg : sel;
    if (kSigMode == 0 && lds_ok) {
      if (s > 0) __syncthreads();   // the previous species' slice is no longer read
      for (int32_t i = tid; i < sg.m; i += kBlock) {
        const double4 q = tb.rec[sg.lo + i];
        sxr[i] = make_double2(q.x, q.w);
        sel[i] = make_double2(q.y, q.z);
      }
      __syncthreads();
    } else if (kSigMode == 3 && lds_ok) {
      // this species' records were fetched into registers while the previous species computed; the next
      // species' go out now and land during this one's lookups
      if (s > 0) __syncthreads();
#pragma unroll
      for (int j = 0; j < kPre; ++j) {
        const int32_t i = tid + j * kBlock;
        if (i < sg.m) {
          sxr[i] = make_double2(pre[j].x, pre[j].w);
          sel[i] = make_double2(pre[j].y, pre[j].z);
        }
      }
      __syncthreads();
      if (s + 1 < NSIG) fetch(s + 1);
    }
    const bool exact = (sg.kind & 4) != 0;
    const double off = tb.offset, chi = tb.chi, nsc = tb.nscale;
    auto emit = [&](int r, double v) {
      const int32_t orow = r0 + r;
      if constexpr (MG) {
        const double cv = chi * v;
        // (TAU: the zero flags are only needed by a phase with non-finite columns; its rows redo them there)
        if constexpr (!TAU) {
          if (!(cv > 0.0)) zb |= 1u << r;
        }
        acc[r] += cv;
      } else {
        if constexpr (TAU) sv[r] = v;
        else if (sig && live && orow < rlim) sig[((int64_t)orow * nse + s) * n_wav + w] = v;
        const double qs = v * nsc;
        acc[r] += qs > 0.0 ? qs : 0.0;
      }
    };
    // the rows' targets first (scalar loads of the Doppler factors, one wait), so that the lookups' LDS reads
    // are not serialised behind them (lgkmcnt counts scalar loads and LDS reads together)
    double tt[R];
#pragma unroll
    for (int r = 0; r < R; ++r) tt[r] = tb.shift[r0 + r < n_rows ? r0 + r : n_rows - 1] * lam;
    if (kSigMode == 2 || !lds_ok) {
      // blocks with a slice too large for LDS (the high-resolution line windows, or a wide spread of Doppler
      // factors): the records straight from the global table (L1 / L2), one 32-byte record per lookup (a second
      // only for lanes whose bracket is the guess +- 1); no guess: the bucket directory (sigma_poly_of)
      if ((sg.kind & 3) > 0) {
        // groups of G rows: G records in flight per lane (the register budget of the LDS path)
        constexpr int G = R < 4 ? R : 4;
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
      // rows past rcap (a problem with fewer rows than R, e.g. one phase shard) are skipped; the guarded
      // copy only runs then (the unguarded one keeps the rows' LDS reads free to overlap)
      auto lds_rows = [&](auto guard) {
        constexpr bool GD = decltype(guard)::value;
        double xk[R];
        double2 el[R];
        if (exact) {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            if (GD && r >= rcap) break;
            const int32_t g = seg_guess(tt[r], sg.xs, sg.inv, sg.m);
            xk[r] = sx_[g].x;
            el[r] = se_[g];
          }
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            if (GD && r >= rcap) break;
            const int32_t g = seg_guess(tt[r], sg.xs, sg.inv, sg.m);
            const double2 xx = sx_[g];
            const int32_t k = tt[r] < xx.x ? g - 1 : (tt[r] >= xx.y ? g + 1 : g);
            xk[r] = sx_[k].x;
            el[r] = se_[k];
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
      if (!TAU && !kSigNoStore && sig && live && orow < rlim) {
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
  __shared__ float2 sqr[TAU ? R * 4 : 1];       // TAU: the (row, half tile) Q ranges
  double etv[TAU ? 4 : 1];
  if constexpr (TAU) {
    // the exp table 2^(i/1024) (the even entries of the 2^(i/2048) table), in flight during the reduction
#pragma unroll
    for (int m = 0; m < 4; ++m) etv[m] = kExp2TableDev[2 * (tid + kBlock * m)];   // kBlock == 256
  }
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
    if constexpr (TAU) {
      if (pp == 0) sqr[r * 4 + h] = q_range(mn, mx);
    } else if (pp == 0 && r0 + r < rlim && hw2 < n_halves) {
      reinterpret_cast<float2*>(tq)[(int64_t)(r0 + r) * n_halves + hw2] = q_range(mn, mx);
    }
  }
  if constexpr (TAU) {
    __syncthreads();   // the Q staging is read: the slices' LDS takes the exp table and the record buffers
    double* sexp = reinterpret_cast<double*>(slds);   // [1024]
#pragma unroll
    for (int m = 0; m < 4; ++m) sexp[tid + kBlock * m] = etv[m];
    __syncthreads();
    constexpr int K = Monos<1>::K;              // tail moments of one effective absorber
    constexpr int RB = 2 * kHeavy;              // record doubles of a light window ({F, N} x <= kHeavy)
    constexpr int WB = R * (RB + K);            // LDS doubles per wavefront: its rows' records and moments
    static_assert(sizeof(double2) * 2 * kSigSeg >= sizeof(double) * (1024 + 4 * WB), "exp table + buffers fit");
    const int hh = __builtin_amdgcn_readfirstlane(tid >> 6);   // this wavefront's half tile of the block
    const int lane = tid & 63;
    double* srb = sexp + 1024 + WB * hh;        // [R][RB] records, then [R][K] moments
    double* smm = srb + R * RB;
    const int64_t tl = wb * 2 + (hh >> 1);                      // its 128-wavelength tile
    const bool live1 = tl * kTW + 64 < n_wav;                   // the tile's second half holds wavelengths
    const bool wave_live = tl < ta.n_tiles && ((hh & 1) == 0 || live1);
    if (wave_live) {
      // (A) lane r < rcap: row r's tile window (k_windows: the union of the tile's halves' Q ranges), flags and
      //     transparent fraction; a heavy row's entry (its own half's window) goes to the lists here
      int32_t wh = 0, wt = 0, wfl = 0;
      double wtf = 0.0;
      if (lane < rcap) {
        const int32_t o = r0 + lane;
        const int32_t* c = ta.counts + o * kCnt;
        const int32_t nact = c[0], nnf = c[3], G = c[4];
        const bool sorted = c[5] != 0, wtab = c[6] != 0;
        wtf = ta.tfrac[o];
        const int32_t pfl = (sorted ? 1 : 0) | (nnf ? 4 : 0);
        const int32_t t_all = sorted ? G : nact;
        const int32_t* hB = ta.wenv + (int64_t)o * 2 * kEnvN;
        const int32_t* hA = hB + kEnvN;
        auto window_of = [&](float ql, float qh, int32_t* hp, int32_t* tp) {
          int32_t h = 0, t = t_all;
          if (wtab && ql >= 0.0f) {
            const int vt = env_floor((float)tail_eps<1>() / qh * (1.0f - 0x1p-20f));
            const int vh = env_floor((float)kTauSat / ql * (1.0f + 0x1p-20f));
            t = vt > kEnvVmax ? 0 : (vt < kEnvVmin ? G : hB[vt - kEnvVmin]);
            h = vh >= kEnvVmax ? 0 : hA[vh + 1 < kEnvVmin ? 0 : vh + 1 - kEnvVmin];
          }
          *hp = h < t ? h : t;
          *tp = t;
        };
        const float2 qa = sqr[lane * 4 + (hh & 2)], qb = sqr[lane * 4 + (hh | 1)];
        const bool bad = qa.x < 0.0f || (live1 && qb.x < 0.0f);
        const float ql = bad ? -1.0f : (live1 ? fminf(qa.x, qb.x) : qa.x);
        const float qh = bad ? 0.0f : (live1 ? fmaxf(qa.y, qb.y) : qa.y);
        window_of(ql, qh, &wh, &wt);
        wfl = pfl | ((wtab && wt < G) ? 2 : 0);
        if (!(wfl & 4) && wt - wh > kHeavy) {
          const float2 qo = sqr[lane * 4 + hh];
          int32_t h2, t2;
          window_of(qo.x, qo.y, &h2, &t2);
          const int32_t ff = pfl | ((wtab && t2 < G) ? 2 : 0);
          const int big = t2 - h2 > kChunk ? 1 : 0;
          const int32_t idx = atomicAdd(&ta.hcnt[big], 1);
          ta.hlist[(big ? ta.hcap : 0) + idx] = make_int4((int32_t)(wb * 4 + hh), h2, t2, ff | (o << 8));
        }
      }
      // (B) the light rows' records and tail moments into the wavefront's LDS, 64 / R lanes per row
      {
        constexpr int LPR = 64 / R;
        const int gr = lane / LPR, j = lane % LPR;
        const int32_t h = __shfl(wh, gr, 64), t = __shfl(wt, gr, 64), fl = __shfl(wfl, gr, 64);
        if (gr < rcap && !(fl & 4) && t - h <= kHeavy) {
          const int32_t o = r0 + gr;
          const double* src = ((fl & 1) ? ta.mrecs : ta.recs) + ((int64_t)o * ta.n_pr + h) * 2;
          for (int e = j; e < 2 * (t - h); e += LPR) srb[gr * RB + e] = src[e];
          if (fl & 2) {
            const double* mp = ta.wmom + ((int64_t)o * (ta.n_pr + 1) + t) * K;
            for (int k = j; k < K; k += LPR) smm[gr * K + k] = mp[k];
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // (C) per row: the light window (k_tau_p's static unit: records in order, the tail polynomial, the
      //     transparent sum), the exact chord-order path, or Y for a heavy half tile's entry
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r >= rcap) break;
        const int32_t o = r0 + r;
        double yv;
        if constexpr (MG) yv = acc[r];
        else yv = sv[r];
        const int32_t h = lane_read(wh, r), t = lane_read(wt, r), fl = lane_read(wfl, r);
        const double tf = lane_read(wtf, r);
        const int32_t n = t - h;
        if (!(fl & 4) && n <= kHeavy) {
          const double* rb = srb + r * RB;
          const double sy = yv * kM1024Ln2;
          double a = 0.0;
          for (int32_t q = 0; q < n; ++q) a = acc_exp1024(a, rb[2 * q], rb[2 * q + 1] * sy, sexp);
          if (fl & 2) {
            double mm[K];
#pragma unroll
            for (int k = 0; k < K; ++k) mm[k] = smm[r * K + k];
            const double qv[1] = {yv * ta.nscale};
            a += tail_eval<1>(mm, qv);
          }
          a += tf;
          if (live) ta.R[(int64_t)o * n_wav + w] = a;
          if (ta.evals) {
            const int nl = __popcll(__ballot(live));
            if (lane == 0) atomicAdd(&ta.evals[(blockIdx.x * 4 + hh) & 63], (unsigned long long)n * (unsigned long long)nl);
          }
        } else if (fl & 4) {
          // non-finite column densities: the reference's chord order with ocml exp
          const double* rb = ta.recs + (int64_t)o * ta.n_pr * 2;
          const int32_t* ipl = ta.act_ip + (int64_t)o * ta.n_pr;
          // merged species: some chi_s sigma_s not > 0 at this (row, wavelength) -- the same records and
          // arithmetic as the lookups above (sigma_seg_poly), so the same values
          bool zr = false;
          if constexpr (MG) {
#pragma unroll
            for (int s = 0; s < NSIG; ++s) {
              const SigTabDev& tb = tabv.t[s];
              const double v = sigma_seg_poly(tb.shift[o] * lam, tb, seg[wb * NSIG + s], pc, D);
              zr = zr || !(tb.chi * v > 0.0);
            }
          }
          double a = 0.0;
          for (int32_t i = 0; i < t; ++i) {
            const double N = rb[2 * i + 1];
            double tau = N * yv;
            if (zr && !__builtin_isfinite(N)) tau = __builtin_nan("");
            a = a + ta.fout[ipl[i]] * exp(-tau);
          }
          const double fs = ta.fsum[o];
          if (live) ta.R[(int64_t)o * n_wav + w] = (a + tf * fs) / fs;
        } else if (live) {
          ta.sigh[(int64_t)o * n_wav + w] = yv;   // heavy: k_tau_p integrates the entry from this row
        }
      }
    }
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
                       int32_t merge_sp, double nscale_m, uint8_t* zfl, hipEvent_t ev_start, hipEvent_t ev_stop,
                       const TauArgs* tau) {
  const int32_t n_blk = (int32_t)grid_for(n_wav);
  // rows per workgroup: PROM_SIG_POLY_ROWS when set at build time, else 8 for several species (their lookups
  // fill the workgroup) and 4 for one (more workgroups in flight)
  const int R = kSigPolyRows > 0 ? kSigPolyRows : (nsig >= 2 ? 8 : 4);
  const int32_t n_rc = (n_rows + R - 1) / R;
  // PROM_SIG_PARTS (profiling builds only, -DPROM_PROFILE_PARTS: R is wrong without both): 1 = LDS
  // workgroups, 2 = global-record ones; the product library always runs both
#ifdef PROM_PROFILE_PARTS
  static const int32_t parts = [] {
    const char* e = std::getenv("PROM_SIG_PARTS");
    const int v = e ? std::atoi(e) : 3;
    return (v >= 1 && v <= 3) ? v : 3;
  }();
#else
  constexpr int32_t parts = 3;
#endif
  // front: the oversize blocks' workgroups; then the XCD-aware grid over all blocks (none when every
  // block is oversize)
  // rows per front workgroup (measured, profiles/r03_sigma_rf_sweep.txt): R / 2 for several species (C3: 4
  // of 8 rows, 37 against 49 us isolated); one species: all R rows when there are >= 16384 (block, row)
  // pairs of oversize blocks (C4x10: 86 against 102 us at R / 2), else R / 2 (C4: 14.3 us, 21.2 at R; a
  // C4x10 eighth shard: 25.5 against 31.6 us) -- PROM_SIG_RF overrides
  static const int rf_env = std::getenv("PROM_SIG_RF") ? std::atoi(std::getenv("PROM_SIG_RF")) : 0;
  int RF = R;
  if (rf_env > 0) RF = rf_env < R ? rf_env : R;
  else if (nsig >= 2 || (int64_t)n_fb * n_rows < 16384) RF = R / 2;
  const int64_t n_front = (int64_t)((n_fb + 7) / 8) * 8 * ((n_rows + RF - 1) / RF);
  const unsigned nb = (unsigned)(n_front + (n_fb >= n_blk ? 0 : (int64_t)((n_blk + 7) / 8) * 8 * n_rc));
  const PolyCoef& pc = poly_coef();
  const TauArgs ta = tau ? *tau : TauArgs{};
  PROM_REQUIRE(!tau || merge_sp || nsig == 1, "fused Doppler rows: one effective absorber only");
#define PROM_SIGK(NS, DG, MGV, RV, TV)                                                                         \
  hipExtLaunchKernelGGL((k_sigma_poly<NS, DG, MGV, RV, TV>), dim3(nb), dim3(kBlock), 0, s, ev_start, ev_stop, 0, \
                        tabv, pc, wav, n_wav, n_rows, seg, fb, n_fb, n_blk, n_rc, sig, tq, merge_sp, nscale_m, zfl, \
                        parts, RF, ta)
  // the fused (TAU) instantiations: merged species (NS >= 2) and one unmerged species (NS == 1)
#define PROM_SIGP(NS, DG, MGT)                                                                                 \
  do {                                                                                                         \
    if (tau) {                                                                                                 \
      if (R == 8) PROM_SIGK(NS, DG, MGT, 8, true); else PROM_SIGK(NS, DG, MGT, 4, true);                     \
    } else if (merge_sp && R == 8) PROM_SIGK(NS, DG, true, 8, false);                                         \
    else if (merge_sp) PROM_SIGK(NS, DG, true, 4, false);                                                      \
    else if (R == 8) PROM_SIGK(NS, DG, false, 8, false);                                                       \
    else PROM_SIGK(NS, DG, false, 4, false);                                                                   \
  } while (0)
#define PROM_SIGP_D(NS, MGT)                 \
  switch (deg) {                             \
    case 4: PROM_SIGP(NS, 4, MGT); break;    \
    case 6: PROM_SIGP(NS, 6, MGT); break;    \
    case 8: PROM_SIGP(NS, 8, MGT); break;    \
    case 10: PROM_SIGP(NS, 10, MGT); break;  \
    case 12: PROM_SIGP(NS, 12, MGT); break;  \
    default: PROM_SIGP(NS, 14, MGT); break;  \
  }
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

// ---- half-tile Q bounds for the fused path (no sigma rows in HBM) -------------------------------------
// k_order / k_windows pick each tile's tau window from a Q range that must enclose Q at every wavelength of
// the half tile.  Without the sigma rows it is bounded from the table nodes the half tile's targets can
// interpolate between: numpy.interp's value lies between its bracket nodes' values, so log10 sigma_s is
// within [min, max] of f over the nodes bracketing the first to the last target (verified guess +- 1
// node), and 10^f - offset is monotone (widened by 2^-50 against the last-ulp behaviour of exp10).  Blocks
// without a verified guess take their whole slice's range; targets outside the table or non-finite give
// the "bad" range (-1, 0): window = every record.  One thread per (row, half tile).
__device__ __forceinline__ void node_range(const double* __restrict__ y, int64_t a, int64_t b, double* lo, double* hi) {
  double mn = y[a], mx = y[a];
  for (int64_t i = a + 1; i <= b; ++i) {
    const double v = y[i];
    mn = v < mn ? v : mn;
    mx = v > mx ? v : mx;
  }
  *lo = mn;
  *hi = mx;
}

template <int NSIG>
__global__ void __launch_bounds__(kBlock) k_qbounds(const SigTabs4 tabv, const double* __restrict__ wav, int64_t n_wav,
                                                  int32_t n_rows, const SigSeg* __restrict__ seg, float4* __restrict__ tq,
                                                  int32_t merge_sp, double nscale_m) {
  const int64_t n_halves = 2 * ((n_wav + kTW - 1) / kTW);
  const int64_t item = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  if (item >= (int64_t)n_rows * n_halves) return;
  const int32_t orow = (int32_t)(item / n_halves);
  const int64_t hw = item - (int64_t)orow * n_halves;
  const int64_t w0 = hw * 64, w1 = (w0 + 63 < n_wav ? w0 + 63 : n_wav - 1);
  const int64_t wb = w0 / kBlock;   // the 256-wavelength block (segments) of this half tile
  bool bad = !(w0 < n_wav);
  double qlo = 0.0, qhi = 0.0, ylo = 0.0, yhi = 0.0;
#pragma unroll
  for (int s = 0; s < NSIG; ++s) {
    const SigTabDev& tb = tabv.t[s];
    const SigSeg sg = seg[wb * NSIG + s];
    double flo, fhi;
    if (sg.m <= 0) { bad = true; continue; }
    const double ta = tb.shift[orow] * wav[w0 < n_wav ? w0 : n_wav - 1], tz = tb.shift[orow] * wav[w1];
    if ((sg.kind & 3) > 0) {
      // first / last target's bracket within one node of the guess: the range [g_a - 1, g_z + 2] holds both
      // brackets' nodes
      const int32_t ga = seg_guess(ta, sg.xs, sg.inv, sg.m), gz = seg_guess(tz, sg.xs, sg.inv, sg.m);
      const int64_t a = (int64_t)sg.lo + (ga > 0 ? ga - 1 : 0);
      const int64_t b = (int64_t)sg.lo + (gz + 2 < sg.m ? gz + 2 : sg.m - 1);
      node_range(tb.y, a, b, &flo, &fhi);
    } else {
      node_range(tb.y, sg.lo, (int64_t)sg.lo + sg.m - 1, &flo, &fhi);
    }
    const double slo = (exp10(flo) - tb.offset) * (1.0 - 0x1p-50), shi = (exp10(fhi) - tb.offset) * (1.0 + 0x1p-50);
    if (merge_sp) {
      ylo += tb.chi * slo;
      yhi += tb.chi * shi;
    } else {
      const double a = slo * tb.nscale, b = shi * tb.nscale;
      qlo += a > 0.0 ? a : 0.0;
      qhi += b > 0.0 ? b : 0.0;
    }
  }
  if (merge_sp) {
    const double a = ylo * nscale_m, b = yhi * nscale_m;
    qlo = a > 0.0 ? a : 0.0;
    qhi = b > 0.0 ? b : 0.0;
  }
  // sums of NSIG terms: relative rounding below 2^-45
  qlo *= 1.0 - 0x1p-45;
  qhi *= 1.0 + 0x1p-45;
  bad = bad || !(qhi <= 1.0e100) || !(qlo == qlo);
  reinterpret_cast<float2*>(tq)[(int64_t)orow * n_halves + hw] =
      bad ? make_float2(-1.0f, 0.0f) : q_range((float)qlo, (float)qhi);
}

void launch_qbounds(hipStream_t s, int32_t nsig, const SigTabs4& tabv, const double* wav, int64_t n_wav, int32_t n_rows,
                    const SigSeg* seg, float4* tq, int32_t merge_sp, double nscale_m) {
  const int64_t n_halves = 2 * ((n_wav + kTW - 1) / kTW);
  const unsigned nb = grid_for((int64_t)n_rows * n_halves);
#define PROM_QB(NS) \
  hipLaunchKernelGGL((k_qbounds<NS>), dim3(nb), dim3(kBlock), 0, s, tabv, wav, n_wav, n_rows, seg, tq, merge_sp, nscale_m)
  switch (nsig) {
    case 1: PROM_QB(1); break;
    case 2: PROM_QB(2); break;
    case 3: PROM_QB(3); break;
    default: PROM_QB(4); break;
  }
#undef PROM_QB
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
