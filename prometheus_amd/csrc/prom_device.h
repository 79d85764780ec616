// Device-side building blocks shared by the kernel translation units (prom_fn.hip, prom_transit.hip,
// prom_mol.hip, prom_rm.hip).  Compiled with -ffp-contract=off: every product and sum is rounded exactly
// where the numpy reference rounds it (no silent FMA contraction); explicit FMAs appear only inside the
// documented exp evaluations and tail polynomials, as in any libm.
#pragma once
#include <hip/hip_ext.h>

#include "exp2_table.h"
#include "faddeeva.h"
#include "prom_internal.h"

namespace prom {

constexpr int kBlock = 256;
constexpr int kTW = 128;   // k_tau_w: wavelengths per workgroup (one window tile)
constexpr int kTP = 4;     // k_tau_w: phases per workgroup (one per wavefront)
constexpr int kHeavy = 8;  // k_tau_p: tiles whose window is longer than this become heavy entries
constexpr int kChunk = 64; // k_tau_p: records per chunk of a heavy entry (longer entries: one workgroup)

// Optional in-kernel timing (build with -DPROM_TRACE, tools/trace_kernels.py): wall-clock stamps
// (100 MHz) of workgroup 0's steps and per-wavefront cycle counters in a device array.
#ifdef PROM_TRACE
static __device__ unsigned long long g_trace[1 << 20];
#define PROM_TS(slot)                                                   \
  do {                                                                  \
    __syncthreads();                                                    \
    if (threadIdx.x == 0) g_trace[(slot)] = wall_clock64();             \
  } while (0)
#define PROM_ACC(slot, v)                                               \
  do {                                                                  \
    if ((threadIdx.x & 63) == 0) g_trace[(slot)] += (unsigned long long)(v); \
  } while (0)
#else
#define PROM_TS(slot) do {} while (0)
#define PROM_ACC(slot, v) do {} while (0)
#endif
#ifdef PROM_TRACE
#define PROM_CLK(var) const long long var = clock64()
#else
#define PROM_CLK(var) do {} while (0)
#endif

static __constant__ double kExp2TableDev[PROM_EXP2_TABLE_N] = {
#define PROM_EXP2_TABLE_BODY
#include "exp2_table_body.h"
};

static inline unsigned grid_for(int64_t n, int block = kBlock, int64_t cap = 1 << 20) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

// numpy.interp (numpy/_core/src/multiarray/compiled_base.c arr_interp) for one target.
__device__ __forceinline__ double np_interp(double t, const double* __restrict__ xp,
                                            const double* __restrict__ fp, int64_t n) {
  if (t != t) return t;
  if (n == 1) return (t < xp[0]) ? fp[0] : fp[0];
  if (t < xp[0]) return fp[0];
  if (t > xp[n - 1]) return fp[n - 1];
  if (t == xp[n - 1]) return fp[n - 1];
  int64_t lo = 0, hi = n - 1;  // xp[lo] <= t < xp[hi]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) >> 1;
    if (xp[mid] <= t) lo = mid; else hi = mid;
  }
  if (xp[lo] == t) return fp[lo];
  const double slope = (fp[lo + 1] - fp[lo]) / (xp[lo + 1] - xp[lo]);
  double r = slope * (t - xp[lo]) + fp[lo];
  if (r != r) {
    r = slope * (t - xp[lo + 1]) + fp[lo + 1];
    if (r != r && fp[lo] == fp[lo + 1]) r = fp[lo];
  }
  return r;
}

// np_interp for one table of a transit problem, then 10^v - offset.  The bracket (numpy's: the largest
// j <= n-2 with xp[j] <= t) comes from the bucket directory: dir[j] - 1 is the last node at or before
// the bucket's start, and a window of 4 nodes (x and f fetched together) holds the bracket unless the
// bucket is crowded or rounding moved j, in which case a gallop + bisection finds it.
__device__ __forceinline__ double sigma_of(double t, const SigTabDev& tb) {
  const double* __restrict__ xp = tb.x;
  const double* __restrict__ fp = tb.y;
  const int64_t n = tb.n;
  double v;
  if (t != t) v = t;
  else if (n == 1 || !(t >= xp[0])) v = fp[0];
  else if (t >= xp[n - 1]) v = fp[n - 1];
  else {
    const double fj = (t - tb.dir_x0) * tb.dir_inv_h;
    const int32_t j = fj < 0.0 ? 0 : (fj >= (double)(tb.n_dir - 1) ? tb.n_dir - 1 : (int32_t)fj);
    int64_t lo = tb.dir[j] - 1;
    lo = lo < 0 ? 0 : (lo > n - 2 ? n - 2 : lo);
    const int64_t l1 = lo + 1, l2 = lo + 2 < n ? lo + 2 : n - 1, l3 = lo + 3 < n ? lo + 3 : n - 1;
    const double x0 = xp[lo], x1 = xp[l1], x2 = xp[l2], x3 = xp[l3];
    const double f0 = fp[lo], f1 = fp[l1], f2 = fp[l2], f3 = fp[l3];
    double xa, xb, fa, fb;
    int64_t k = -1;
    if (x0 <= t) {
      if (t < x1) { k = lo; xa = x0; xb = x1; fa = f0; fb = f1; }
      else if (t < x2) { k = l1; xa = x1; xb = x2; fa = f1; fb = f2; }
      else if (t < x3) { k = l2; xa = x2; xb = x3; fa = f2; fb = f3; }
    }
    if (k < 0) {
      int64_t a = lo, b = l3;   // invariant after the gallop: xp[a] <= t < xp[b]
      for (int64_t st = 1; a > 0 && xp[a] > t; st <<= 1) { b = a; a = a - st > 0 ? a - st : 0; }
      for (int64_t st = 1; b < n - 1 && xp[b] <= t; st <<= 1) { a = b; b = b + st < n - 1 ? b + st : n - 1; }
      while (b - a > 1) {
        const int64_t mid = (a + b) >> 1;
        if (xp[mid] <= t) a = mid; else b = mid;
      }
      k = a;
      xa = xp[a]; xb = xp[a + 1]; fa = fp[a]; fb = fp[a + 1];
    }
    if (xa == t) v = fa;
    else {
      const double slope = (fb - fa) / (xb - xa);
      v = slope * (t - xa) + fa;
      if (v != v) {
        v = slope * (t - xb) + fb;
        if (v != v && fa == fb) v = fa;
      }
    }
  }
  return exp10(v) - tb.offset;
}

// numpy.interp of one target from its bracket guess g (within one node of the bracket, SigSeg): x_g and
// x_{g+1} decide between g - 1, g and g + 1, then the bracket's record {x, f, slope} gives the value --
// two dependent reads, no branches on the common path.  X2(g) reads x_g and x_{g+1}, REC(k, ...) node k's
// x, f and slope.
template <class XF, class RF>
__device__ __forceinline__ double interp_guess(double t, int32_t g, XF X2, RF REC) {
  const double2 xg = X2(g);   // x_g, x_{g+1}
  const int32_t k = t < xg.x ? g - 1 : (t >= xg.y ? g + 1 : g);
  double xa, fa, sl;
  REC(k, xa, fa, sl);
  // numpy: an exact node hit returns f; with a finite slope sl (t - x) + f is that f already, so the
  // test is only needed where the interpolation is NaN (non-finite slope), as is numpy's right-node retry
  double rv = sl * (t - xa) + fa;
  if (rv != rv) {
    if (xa == t) rv = fa;
    else {
      double xb, fb, sb;
      REC(k + 1, xb, fb, sb);
      rv = sl * (t - xb) + fb;
      if (rv != rv && fa == fb) rv = fa;
    }
  }
  return rv;
}

__device__ __forceinline__ int32_t seg_guess(double t, double b, double inv, int32_t m) {
  // f = fma(t, inv, b) (b = -x_lo inv), g = (f < 0 ? 0 : f >= m - 2 ? m - 2 : (int)f): the host's verified
  // map (prom_api.hip sigma segments).  Every target lies in the slice, so f is within rounding of
  // [0, m - 1] and truncating first, clamping the integer after, gives the same g
  const int32_t g = (int32_t)__builtin_fma(t, inv, b);
  return max(min(g, m - 2), 0);   // (one v_med3_i32; m >= 2)
}

struct InvFact {
  double v[16];
  constexpr InvFact() : v{} {
    double f = 1.0;
    v[0] = 1.0;
    for (int i = 1; i < 16; ++i) {
      f *= (double)i;
      v[i] = 1.0 / f;
    }
  }
};

// the coefficients travel as a kernel argument (scalar registers: each FMA takes its addend from an SGPR
// pair; as compile-time constants the compiler re-materialises both halves into VGPRs before every use)
struct PolyCoef {
  double c[16];
};

template <int D>
__device__ __forceinline__ double exp_taylor(double a, const PolyCoef& pc) {
  double p = pc.c[D];
#pragma unroll
  for (int k = D - 1; k >= 0; --k) p = __builtin_fma(p, a, pc.c[k]);
  return p;
}

// exp_taylor at a run-time degree (one uniform branch; the degrees launch_sigma_poly instantiates)
__device__ __forceinline__ double exp_taylor_d(double a, const PolyCoef& pc, int32_t deg) {
  switch (deg) {
    case 4: return exp_taylor<4>(a, pc);
    case 6: return exp_taylor<6>(a, pc);
    case 8: return exp_taylor<8>(a, pc);
    case 10: return exp_taylor<10>(a, pc);
    case 12: return exp_taylor<12>(a, pc);
    default: return exp_taylor<14>(a, pc);
  }
}

// the Taylor coefficients 1 / k! (host side, for the kernel arguments)
inline const PolyCoef& poly_coef() {
  static const PolyCoef pc = [] {
    PolyCoef c{};
    constexpr InvFact F{};
    for (int k = 0; k < 16; ++k) c.c[k] = F.v[k];
    return c;
  }();
  return pc;
}

// sigma_s(t) for the fused Doppler path (no sigma rows in HBM): the verified linear guess of the target's
// 256-wavelength block (SigSeg, kind > 0) and two dependent reads of the global x / f arrays (numpy's slope
// divided here), else the directory lookup.  Bit for bit the value k_sigma_rows would have stored.
__device__ __forceinline__ double sigma_seg(double t, const SigTabDev& tb, const SigSeg& sg) {
  if ((sg.kind & 3) > 0) {
    const double* __restrict__ gx = tb.x + sg.lo;
    const double* __restrict__ gy = tb.y + sg.lo;
    const int32_t g = seg_guess(t, sg.xs, sg.inv, sg.m);
    return exp10(interp_guess(
               t, g, [&](int32_t i) { return make_double2(gx[i], gx[i + 1]); },
               [&](int32_t i, double& x, double& f, double& sl) {
                 x = gx[i]; f = gy[i];
                 sl = (gy[i + 1] - f) / (gx[i + 1] - x);
               })) - tb.offset;
  }
  return sigma_of(t, tb);
}

// numpy's bracket of t (the largest j <= n-2 with x_j <= t) for x_0 <= t < x_{n-1}, n >= 2: sigma_of's
// search (bucket directory, 4-node window, gallop + bisection), x only.
__device__ __forceinline__ int64_t bracket_of(double t, const SigTabDev& tb) {
  const double* __restrict__ xp = tb.x;
  const int64_t n = tb.n;
  const double fj = (t - tb.dir_x0) * tb.dir_inv_h;
  const int32_t j = fj < 0.0 ? 0 : (fj >= (double)(tb.n_dir - 1) ? tb.n_dir - 1 : (int32_t)fj);
  int64_t lo = tb.dir[j] - 1;
  lo = lo < 0 ? 0 : (lo > n - 2 ? n - 2 : lo);
  const int64_t l1 = lo + 1, l2 = lo + 2 < n ? lo + 2 : n - 1, l3 = lo + 3 < n ? lo + 3 : n - 1;
  const double x0 = xp[lo], x1 = xp[l1], x2 = xp[l2], x3 = xp[l3];
  if (x0 <= t) {
    if (t < x1) return lo;
    if (t < x2) return l1;
    if (t < x3) return l2;
  }
  int64_t a = lo, b = l3;   // invariant after the gallop: xp[a] <= t < xp[b]
  for (int64_t st = 1; a > 0 && xp[a] > t; st <<= 1) { b = a; a = a - st > 0 ? a - st : 0; }
  for (int64_t st = 1; b < n - 1 && xp[b] <= t; st <<= 1) { a = b; b = b + st < n - 1 ? b + st : n - 1; }
  while (b - a > 1) {
    const int64_t mid = (a + b) >> 1;
    if (xp[mid] <= t) a = mid; else b = mid;
  }
  return a;
}

// sigma_s(t) on the polynomial path without a verified guess: the bracket from the directory search, then
// the record's E_k e^(L_k (t - x_k)) - offset -- the value the guessed paths give, so a row does not
// depend on which segment kind a block got (phase shards change the segments: bitwise equal R rows);
// numpy's end rules outside the table (node 0 / n-1: E - offset), NaN in, NaN out.
__device__ __forceinline__ double sigma_poly_of(double t, const SigTabDev& tb, const PolyCoef& pc, int32_t deg) {
  if (t != t) return t;
  const int64_t n = tb.n;
  if (n == 1 || !(t >= tb.x[0])) return __builtin_fma(tb.rec[0].y, 1.0, -tb.offset);
  if (t >= tb.x[n - 1]) return __builtin_fma(tb.rec[n - 1].y, 1.0, -tb.offset);
  const double4 q = tb.rec[bracket_of(t, tb)];
  return __builtin_fma(q.y, exp_taylor_d(q.z * (t - q.x), pc, deg), -tb.offset);
}

// sigma_s(t) on the polynomial path (TransitDev::sig_deg > 0): the block's verified guess, the bracket's
// record {x_k, 10^f_k, ln10 slope_k, x_k+1} (a second record only when the guess is one node off), the
// degree-deg Taylor e^a -- bit for bit the value k_sigma_poly stores (its LDS and global paths read the
// same record); no guess: sigma_poly_of, as there.
__device__ __forceinline__ double sigma_seg_poly(double t, const SigTabDev& tb, const SigSeg& sg, const PolyCoef& pc,
                                                 int32_t deg) {
  if ((sg.kind & 3) > 0) {
    const double4* __restrict__ rr = tb.rec + sg.lo;
    const int32_t g = seg_guess(t, sg.xs, sg.inv, sg.m);
    double4 q = rr[g];
    if (!(sg.kind & 4)) {
      const int32_t k = t < q.x ? g - 1 : (t >= q.w ? g + 1 : g);
      if (k != g) q = rr[k];
    }
    return __builtin_fma(q.y, exp_taylor_d(q.z * (t - q.x), pc, deg), -tb.offset);
  }
  return sigma_poly_of(t, tb, pc, deg);
}

// sigma_of for NS tables at once (the species of one wavelength): every table's directory load goes
// out first, then every table's 4-node window (x and f, 64 B per target: the resampling kernel is bound
// by the vector L1's bytes, so numpy.interp's slope is divided here rather than fetched), so a thread
// waits for two dependent round trips instead of 2 NS.  Same bracket rules and arithmetic as sigma_of, so
// the results are identical bit for bit.
// (TB(s): the table of element s -- tabv.t[s] for a wavelength's species, one table for several targets)
template <int NS, class TB>
__device__ __forceinline__ void sigma_multi_f(TB tbf, const double (&t)[NS], double (&v)[NS]) {
  int32_t d[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const SigTabDev& tb = tbf(s);
    const double fj = (t[s] - tb.dir_x0) * tb.dir_inv_h;
    const int32_t j = fj >= 0.0 ? (fj >= (double)(tb.n_dir - 1) ? tb.n_dir - 1 : (int32_t)fj) : 0;
    d[s] = tb.dir[j];
  }
  struct Win { double x0, x1, x2, x3, f0, f1, f2, f3; } u[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const SigTabDev& tb = tbf(s);
    const int32_t n = (int32_t)tb.n;
    int32_t l = d[s] - 1;
    l = l > n - 2 ? n - 2 : l;
    l = l < 0 ? 0 : l;   // (n == 1: 0)
    const int32_t l1 = l + 1 < n ? l + 1 : n - 1, l2 = l + 2 < n ? l + 2 : n - 1, l3 = l + 3 < n ? l + 3 : n - 1;
    u[s].x0 = tb.x[l]; u[s].x1 = tb.x[l1]; u[s].x2 = tb.x[l2]; u[s].x3 = tb.x[l3];
    u[s].f0 = tb.y[l]; u[s].f1 = tb.y[l1]; u[s].f2 = tb.y[l2]; u[s].f3 = tb.y[l3];
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const SigTabDev& tb = tbf(s);
    const double tt = t[s];
    const bool found = tb.n >= 2 && tt >= tb.xfirst && tt < tb.xlast && u[s].x0 <= tt && tt < u[s].x3;
    const bool c0 = tt < u[s].x1, c1 = tt < u[s].x2;
    const double xa = c0 ? u[s].x0 : (c1 ? u[s].x1 : u[s].x2);
    const double xb = c0 ? u[s].x1 : (c1 ? u[s].x2 : u[s].x3);
    const double fa = c0 ? u[s].f0 : (c1 ? u[s].f1 : u[s].f2);
    const double fb = c0 ? u[s].f1 : (c1 ? u[s].f2 : u[s].f3);
    double r;
    if (xa == tt) r = fa;
    else {
      const double slope = (fb - fa) / (xb - xa);
      r = slope * (tt - xa) + fa;
    }
    if (found && r == r) v[s] = exp10(r) - tb.offset;
    else v[s] = sigma_of(tt, tb);
  }
}

template <int NS>
__device__ __forceinline__ void sigma_multi(const SigTabs4& tabv, const double (&t)[NS], double (&v)[NS]) {
  sigma_multi_f<NS>([&](int s) -> const SigTabDev& { return tabv.t[s]; }, t, v);
}

// ---- wavefront scans on DPP row shifts + cross-row readlanes (no LDS traffic, no bpermute) ----
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xf, 0xf, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
template <int CTRL>
__device__ __forceinline__ int32_t dpp_mov(int32_t v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ double lane_read(double v, int l) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ int32_t lane_read(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

// op over all 64 lanes of a float (every lane active), on DPP moves and four readlanes: no LDS traffic
template <int CTRL>
__device__ __forceinline__ float dpp_movf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <typename Op>
__device__ __forceinline__ float wave_reduce_f(float v, Op op) {
  v = op(v, dpp_movf<0xB1>(v));    // quad_perm [1,0,3,2]
  v = op(v, dpp_movf<0x4E>(v));    // quad_perm [2,3,0,1]
  v = op(v, dpp_movf<0x141>(v));   // row_half_mirror
  v = op(v, dpp_movf<0x140>(v));   // row_mirror
  const float a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float b = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float c = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float d = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return op(op(a, b), op(c, d));
}

// inclusive prefix over lanes 0..63 (op applied as op(earlier, later))
template <typename T, typename Op>
__device__ __forceinline__ T wave_prefix(T v, Op op) {
  const int lane = threadIdx.x & 63, rl = lane & 15, row = lane >> 4;
  T t = dpp_mov<0x111>(v);
  if (rl >= 1) v = op(t, v);
  t = dpp_mov<0x112>(v);
  if (rl >= 2) v = op(t, v);
  t = dpp_mov<0x114>(v);
  if (rl >= 4) v = op(t, v);
  t = dpp_mov<0x118>(v);
  if (rl >= 8) v = op(t, v);
  const T r0 = lane_read(v, 15), r1 = lane_read(v, 31), r2 = lane_read(v, 47);
  const T c01 = op(r0, r1), c012 = op(c01, r2);
  if (row == 1) v = op(r0, v);
  else if (row == 2) v = op(c01, v);
  else if (row == 3) v = op(c012, v);
  return v;
}
// inclusive suffix over lanes 63..0 (op applied as op(earlier, later))
template <typename T, typename Op>
__device__ __forceinline__ T wave_suffix(T v, Op op) {
  const int lane = threadIdx.x & 63, rl = lane & 15, row = lane >> 4;
  T t = dpp_mov<0x101>(v);
  if (rl <= 14) v = op(v, t);
  t = dpp_mov<0x102>(v);
  if (rl <= 13) v = op(v, t);
  t = dpp_mov<0x104>(v);
  if (rl <= 11) v = op(v, t);
  t = dpp_mov<0x108>(v);
  if (rl <= 7) v = op(v, t);
  const T r1 = lane_read(v, 16), r2 = lane_read(v, 32), r3 = lane_read(v, 48);
  const T c23 = op(r2, r3), c123 = op(r1, c23);
  if (row == 2) v = op(v, r3);
  else if (row == 1) v = op(v, c23);
  else if (row == 0) v = op(v, c123);
  return v;
}

// numpy.heaviside(d, 1.0)
__device__ __forceinline__ double heaviside1(double d) { return d < 0.0 ? 0.0 : (d >= 0.0 ? 1.0 : d); }

// One density sample, in the reference's evaluation order (see prom_density_kind in prom_hip.h).
__device__ __forceinline__ double density_at(const DensityDev& m, double xv, double y, double z,
                                             double bx, double by) {
  const double dx = xv - bx, dy = y - by;
  switch (m.kind) {
    case PROM_DENSITY_BAROMETRIC: {
      const double r = sqrt((dx * dx + dy * dy) + z * z);
      return (m.p[0] * exp((m.p[1] - r) / m.p[2])) * heaviside1(r - m.p[1]);
    }
    case PROM_DENSITY_HYDROSTATIC: {
      const double r = sqrt((dx * dx + dy * dy) + z * z);
      const double jeans = m.p[2] / (m.p[3] * r) * heaviside1(r - m.p[1]);
      return m.p[0] * exp(jeans - m.p[4]);
    }
    case PROM_DENSITY_POWERLAW: {
      const double r = sqrt((dx * dx + dy * dy) + z * z);
      const double xr = m.p[1] / r;
      double pw;
      if (m.pad > 0) {
        // x^q for an integral q <= 8 by binary exponentiation (q uniform): at most 2 log2(q) rounded products,
        // within ~8 ulp of numpy's pow (gasProperties.py:241 (R/r)**q)
        pw = 1.0;
        double b = xr;
        for (int32_t e = m.pad - 1; e > 0; e >>= 1) {
          if (e & 1) pw *= b;
          if (e > 1) b *= b;
        }
      } else {
        pw = pow(xr, m.p[2]);
      }
      return (m.p[0] * pw) * heaviside1(r - m.p[1]);
    }
    case PROM_DENSITY_TORUS: {
      const double a = sqrt(dx * dx + dy * dy);
      const double ta = (a - m.p[1]) / m.p[2];
      const double tz = z / m.p[3];
      return m.p[0] * (exp(-(ta * ta)) * exp(-(tz * tz)));
    }
    default:
      return __builtin_nan("");
  }
}

// numpy pairwise_sum of (a[i] * chi) for i < n (numpy/_core/src/umath/loops_utils.h.src),
// then the reduction identity: 0.0 + result.
__device__ __forceinline__ double pw_leaf(const double* __restrict__ a, int64_t n, double chi) {
  if (n < 8) {
    double r = 0.0;
    for (int64_t i = 0; i < n; ++i) r += a[i] * chi;
    return r;
  }
  double r0 = a[0] * chi, r1 = a[1] * chi, r2 = a[2] * chi, r3 = a[3] * chi;
  double r4 = a[4] * chi, r5 = a[5] * chi, r6 = a[6] * chi, r7 = a[7] * chi;
  int64_t i = 8;
  const int64_t lim = n - (n % 8);
  for (; i < lim; i += 8) {
    r0 += a[i + 0] * chi; r1 += a[i + 1] * chi; r2 += a[i + 2] * chi; r3 += a[i + 3] * chi;
    r4 += a[i + 4] * chi; r5 += a[i + 5] * chi; r6 += a[i + 6] * chi; r7 += a[i + 7] * chi;
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += a[i] * chi;
  return res;
}

__device__ double pairwise_sum_chi(const double* __restrict__ a, int64_t n, double chi) {
  if (n <= 128) return 0.0 + pw_leaf(a, n, chi);
  struct Frame { int64_t off, n; int stage; double left; };
  Frame st[48];
  int sp = 0;
  st[0] = {0, n, 0, 0.0};
  double ret = 0.0;
  while (sp >= 0) {
    Frame& f = st[sp];
    if (f.n <= 128) { ret = pw_leaf(a + f.off, f.n, chi); --sp; continue; }
    int64_t n2 = f.n / 2;
    n2 -= n2 % 8;
    if (f.stage == 0) { f.stage = 1; st[++sp] = {f.off, n2, 0, 0.0}; }
    else if (f.stage == 1) { f.left = ret; f.stage = 2; st[++sp] = {f.off + n2, f.n - n2, 0, 0.0}; }
    else { ret = f.left + ret; --sp; }
  }
  return 0.0 + ret;
}

// ---- windowed integration: per-phase record order, envelopes, threshold tables, tail moments ----
// For one phase and one wavelength, tau_i = sum_s N_si sigma_s.  With n_si = c_s N_si (c_s = 1 /
// (chi_s n_ref L): n_ref bounds the scenario's density, L = n_x dx, so n <= 1; SigTabDev::ncoef) and
// q_s = sigma_s / c_s, every record i satisfies
//     a_i Q <= tau_i <= b_i Q,   a_i = min_s n_si,  b_i = max_s n_si,  Q = sum_s q_s
// (sigma_s >= 0 up to the 1e-50 table offset's rounding, which the bounds absorb).
// Records are ordered by b descending (ties: chord index), equal-column chords merged, and two
// envelopes kept: B_i = max_{j >= i} b_j and A_i = min_{j <= i} a_j (both non-increasing in i).
// For a wavefront whose wavelengths have Q in [Q_lo, Q_hi]:
//   * records j >= t with B_t Q_hi < eps have tau_j < eps: their sum of F e^-tau is the cubic Taylor
//     polynomial sum_e q^e M_e(t), with suffix moments M_e(t) = c_e sum_{j >= t} F_j prod_s n_sj^e_s
//     (|e| <= 3, c_e = (-1)^|e| / prod e_s!); truncation error <= eps^4/24 per unit weight;
//   * records j < h with A_h Q_lo >= tau_sat have tau_j >= tau_sat: skipped, error <= e^-tau_sat each;
//   * records h <= j < t are integrated exactly (table exp).
// eps = 2^-10, tau_sat = 40: |dR| <= 2^-40/24 + e^-40 < 4e-14 (merging adds <= 2^-40/e).
// t and h come from per-phase tables indexed by the threshold's binade and top three mantissa bits
// (X_v = the double with bits v << 49): tab_t[v] = #{i : B_i >= X_v}, tab_h[v] = #{i : A_i >= X_v};
// the tau kernel picks the conservative neighbour (X_v <= eps/Q_hi for t, X_v > tau_sat/Q_lo for h).
constexpr int kWBlock = 512;
constexpr int kWPer = kWinMax / kWBlock;           // sorted positions per thread
constexpr int kEnvVmax = 8184;                     // bits(1.0) >> 49
constexpr int kEnvVmin = kEnvVmax - kEnvN + 1;     // X_vmin = 2^-(kEnvN / 8)
// Tail of the window (records with tau < eps at every wavelength of the wavefront): the Taylor
// polynomial of degree D in q_s over suffix moments, truncation <= eps^(D+1)/(D+1)! per unit weight.
// One effective species (NS == 1, e.g. merged species): D = 7, eps = 2^-4 (5.8e-15); otherwise
// D = 3, eps = 2^-10 (3.5e-14) -- (NS+D choose D) moments per record either way stays small.
template <int NS> struct TailDeg { static constexpr int D = NS == 1 ? 7 : 3; };
template <int NS> __host__ __device__ constexpr double tail_eps() { return NS == 1 ? 0x1p-4 : 0x1p-10; }

// histogram slot of a non-negative envelope value: 1 + (table index of its 1/8-octave bucket), 0 below
// the table, kEnvN + 1 above it.  v >= X_e  <=>  (bits(v) >> 49) >= kEnvVmin + e.
__device__ __forceinline__ int32_t env_slot(double v) {
  const int64_t b = (int64_t)(__builtin_bit_cast(unsigned long long, v) >> 49) - kEnvVmin;
  return b < 0 ? 0 : (b >= kEnvN ? kEnvN + 1 : (int32_t)b + 1);
}
constexpr double kTauSat = 40.0;

// Table index of a positive float threshold: the largest v with X_v = double(bits v << 49) <= x;
// below the table for zero/denormal x, above it for +inf.
__device__ __forceinline__ int env_floor(float x) {
  if (!(x >= 1.17549435e-38f)) return -(1 << 28);
  if (!(x <= 3.40282347e+38f)) return 1 << 28;
  return (int)(__builtin_bit_cast(uint32_t, x) >> 20) + 7168;
}


__host__ __device__ constexpr int binom_c(int n, int k) {
  int r = 1;
  for (int i = 1; i <= k; ++i) r = r * (n - k + i) / i;
  return r;
}

// Monomials of total degree <= D in NS variables, by degree then lexicographically; c[k] = (-1)^j / prod e_s!
template <int NS>
struct Monos {
  static constexpr int D = TailDeg<NS>::D;
  static constexpr int K = binom_c(NS + D, D);
  int e[K][NS];
  double c[K];
  constexpr Monos() : e{}, c{} {
    int total = 1;
    for (int s = 0; s < NS; ++s) total *= D + 1;
    int k = 0;
    for (int j = 0; j <= D; ++j)
      for (int idx = 0; idx < total; ++idx) {
        int d[NS] = {};
        int r = idx, sum = 0;
        for (int s = NS - 1; s >= 0; --s) { d[s] = r % (D + 1); r /= D + 1; sum += d[s]; }
        if (sum != j) continue;
        double f = 1.0;
        for (int s = 0; s < NS; ++s) {
          e[k][s] = d[s];
          for (int m = 2; m <= d[s]; ++m) f *= m;
        }
        c[k] = ((j & 1) ? -1.0 : 1.0) / f;
        ++k;
      }
  }
};

// p[s][j] = v_s^j, formed as ((v v) v) ...
template <int NS>
__device__ __forceinline__ void tail_pows(const double (&v)[NS], double (&p)[NS][TailDeg<NS>::D + 1]) {
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    p[s][0] = 1.0;
    p[s][1] = v[s];
#pragma unroll
    for (int j = 2; j <= TailDeg<NS>::D; ++j) p[s][j] = p[s][j - 1] * v[s];
  }
}

// prod_s p[s][e_s] for monomial k
template <int NS>
__device__ __forceinline__ double mono_eval(const Monos<NS>& M, int k, const double (&p)[NS][TailDeg<NS>::D + 1]) {
  double r = 1.0;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (M.e[k][s]) r *= p[s][M.e[k][s]];
  return r;
}

// The tail sum_k mm[k] q^e_k (mm already carries c[k]): Horner for one species, monomials otherwise.
// Every tau kernel evaluates it through this function, so they agree bit for bit.
template <int NS>
__device__ __forceinline__ double tail_eval(const double (&mm)[Monos<NS>::K], const double (&q)[NS]) {
  constexpr Monos<NS> M{};
  constexpr int K = Monos<NS>::K;
  if constexpr (NS == 1) {
    double tl = mm[K - 1];
#pragma unroll
    for (int k = K - 2; k >= 0; --k) tl = __builtin_fma(tl, q[0], mm[k]);
    return tl;
  } else {
    double p[NS][TailDeg<NS>::D + 1];
    tail_pows<NS>(q, p);
    double tl = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) tl = __builtin_fma(mm[k], mono_eval<NS>(M, k, p), tl);
    return tl;
  }
}

struct OpAdd { template <typename T> __device__ T operator()(T a, T b) const { return a + b; } };
struct OpMax { __device__ double operator()(double a, double b) const { return a > b ? a : b; } };
struct OpMin { __device__ double operator()(double a, double b) const { return a < b ? a : b; } };

// Workgroup barrier for LDS data only: waits for this wave's LDS operations (lgkmcnt), not for its global
// loads and stores (HIP's __syncthreads fences every address space: vmcnt(0) before the barrier, so a
// wave's outstanding global stores would stall the whole workgroup at every step)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Exclusive scans over the kWBlock threads of a workgroup (8 waves); wsum: NW slots of LDS.
// *total (optional) receives the fold over all threads.
template <typename T, typename Op>
__device__ __forceinline__ T wg_excl_prefix(T v, Op op, T id, T* wsum, T* total = nullptr) {
  constexpr int NW = kWBlock / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T inc = v;
  for (int off = 1; off < 64; off <<= 1) {
    const T u = __shfl_up(inc, off, 64);
    if (lane >= off) inc = op(inc, u);
  }
  T exc = __shfl_up(inc, 1, 64);
  if (lane == 0) exc = id;
  lds_barrier();
  if (lane == 63) wsum[wid] = inc;
  lds_barrier();
  T carry = id, all = id;
  for (int w = 0; w < NW; ++w) {
    if (w < wid) carry = op(carry, wsum[w]);
    all = op(all, wsum[w]);
  }
  if (total) *total = all;
  return op(carry, exc);
}

template <typename T, typename Op>
__device__ __forceinline__ T wg_excl_suffix(T v, Op op, T id, T* wsum) {
  constexpr int NW = kWBlock / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T inc = v;
  for (int off = 1; off < 64; off <<= 1) {
    const T u = __shfl_down(inc, off, 64);
    if (lane + off < 64) inc = op(inc, u);
  }
  T exc = __shfl_down(inc, 1, 64);
  if (lane == 63) exc = id;
  __syncthreads();
  if (lane == 0) wsum[wid] = inc;
  __syncthreads();
  T carry = id;
  for (int w = NW - 1; w > wid; --w) carry = op(carry, wsum[w]);
  return op(carry, exc);
}

// tau of one chord in the exact (non-finite column) path.  With merged species (zf != nullptr) the
// single column is N = dx sum_x n and Y = sum_s chi_s sigma_s: the reference's sum_s (N chi_s) sigma_s is
// NaN for an infinite N wherever some chi_s sigma_s is not > 0 (zf[w]), which N Y alone would miss.
__device__ __forceinline__ double exact_tau_merged(double N, double Y, const uint8_t* __restrict__ zf, int64_t w) {
  double tau = N * Y;
  if (zf && !__builtin_isfinite(N) && zf[w]) tau = __builtin_nan("");
  return tau;
}

// ---- fast exp: acc + F * 2^(y/2048) with a 2048-entry table in LDS --------------------------------
// y = -tau * 2048/ln2.  k = rint(y), d = y - k in [-1/2, 1/2],
//   2^(y/2048) = 2^(k >> 11) * T[k & 2047] * exp(d ln2/2048),
// exp(d c) = 1 + d (c + d (c^2/2 + d c^3/6)) with c = ln2/2048: truncation (c/2)^4/24 = 3.5e-17.
// Finite y only (non-finite column densities take the exact path); y below -2^31 saturates the
// integer conversion and ldexp flushes the term to 0, which is exp's own answer there.
constexpr double kExpC1 = 0.0003384507717577858;     // ln2 / 2048
constexpr double kExpC2 = 5.727446245172041e-08;     // c^2 / 2
constexpr double kExpC3 = 6.461528672932366e-12;     // c^3 / 6
constexpr double kMinus2048OverLn2 = -2954.639443740597;

__device__ __forceinline__ double acc_exp2k(double acc, double F, double y, const double* __restrict__ tab) {
  const double k = __builtin_rint(y);
  const int ki = (int)k;
  const double d = y - k;
  double t = __builtin_fma(d, kExpC3, kExpC2);
  t = __builtin_fma(d, t, kExpC1);
  const double e = __builtin_fma(d, t, 1.0);
  const double S = __builtin_amdgcn_ldexp(tab[ki & (PROM_EXP2_TABLE_N - 1)], ki >> 11);
  return __builtin_fma(F * S, e, acc);
}

// acc + F * exp(-tau) with y = -tau * 256 / ln2 given: 2^(y/256) = 2^(k >> 8) T[k & 255] exp(d ln2/256),
// k = rint(y), d = y - k in [-1/2, 1/2], degree-5 Taylor polynomial (truncation (ln2/512)^6/720 = 9e-21
// relative), T[i] = 2^(i/256) = the 2048-entry table at 8i (LDS, 2 KB).  y below -2^31 saturates the
// integer conversion and ldexp returns 0, exp's own answer there.  About 12 FP64 operations.
constexpr double kE256C1 = 0x1.62e42fefa39efp-9;   // (ln2/256)^1 / 1!
constexpr double kE256C2 = 0x1.ebfbdff82c58fp-19;  // (ln2/256)^2 / 2!
constexpr double kE256C3 = 0x1.c6b08d704a0c0p-29;  // (ln2/256)^3 / 3!
constexpr double kE256C4 = 0x1.3b2ab6fba4e77p-39;  // (ln2/256)^4 / 4!
constexpr double kE256C5 = 0x1.5d87fe78a6731p-50;  // (ln2/256)^5 / 5!
constexpr double kM256Ln2 = -0x1.71547652b82fep+8; // -256 / ln2

__device__ __forceinline__ double acc_exp256(double acc, double F, double y, const double* __restrict__ tab) {
  const double k = __builtin_rint(y);
  const int ki = (int)k;
  const double d = y - k;
  double p = __builtin_fma(d, kE256C5, kE256C4);
  p = __builtin_fma(d, p, kE256C3);
  p = __builtin_fma(d, p, kE256C2);
  p = __builtin_fma(d, p, kE256C1);
  p = __builtin_fma(d, p, 1.0);
  const double S = __builtin_amdgcn_ldexp(tab[ki & 255], ki >> 8);
  return __builtin_fma(F * S, p, acc);
}

// acc + F * exp(-tau) with y = -tau * 1024 / ln2 given: 2^(y/1024) = 2^(k >> 10) T[k & 1023] exp(d ln2/1024),
// k = rint(y), d in [-1/2, 1/2], cubic Taylor polynomial (truncation (ln2/2048)^4/24 = 5.5e-16 relative),
// T[i] = 2^(i/1024) = the 2048-entry table at 2i (LDS, 8 KB).  About 10 FP64 operations.
constexpr double kE1024C1 = 0x1.62e42fefa39efp-11;  // (ln2/1024)^1 / 1!
constexpr double kE1024C2 = 0x1.ebfbdff82c58fp-23;  // (ln2/1024)^2 / 2!
constexpr double kE1024C3 = 0x1.c6b08d704a0c0p-35;  // (ln2/1024)^3 / 3!
constexpr double kM1024Ln2 = -0x1.71547652b82fep+10; // -1024 / ln2

__device__ __forceinline__ double acc_exp1024(double acc, double F, double y, const double* __restrict__ tab) {
  const double k = __builtin_rint(y);
  const int ki = (int)k;
  const double d = y - k;
  double p = __builtin_fma(d, kE1024C3, kE1024C2);
  p = __builtin_fma(d, p, kE1024C1);
  p = __builtin_fma(d, p, 1.0);
  const double S = __builtin_amdgcn_ldexp(tab[ki & 1023], ki >> 10);
  return __builtin_fma(F * S, p, acc);
}

__device__ __forceinline__ void fill_exp_table(double* etab) {
  for (int i = threadIdx.x; i < PROM_EXP2_TABLE_N; i += kBlock) etab[i] = kExp2TableDev[i];
}

// ------------------------------------------------------------------ molecular lookup
// Bracketing index of a sorted axis for RegularGridInterpolator (scipy _find_indices):
// i = searchsorted(g, v) - 1 clipped to [0, n-2]; t = (v - g[i]) / (g[i+1] - g[i]).
// Returns false when v is outside [g[0], g[n-1]] (fill value).
__device__ __forceinline__ bool rgi_bracket(const double* __restrict__ g, int64_t n, double v, int64_t* i,
                                            double* t) {
  if (!(v >= g[0] && v <= g[n - 1])) return false;
  int64_t lo = 0, hi = n;  // first index with g[idx] >= v  (searchsorted left)
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (g[mid] < v) lo = mid + 1; else hi = mid;
  }
  int64_t k = lo - 1;
  if (k < 0) k = 0;
  if (k > n - 2) k = n - 2;
  *i = k;
  *t = (v - g[k]) / (g[k + 1] - g[k]);
  return true;
}

// Trilinear value at (P, T, w), scipy's hypercube order: corners (dP, dT, dw) lexicographic,
// weight = ((1 * wP) * wT) * ww, value = ((0 + v000 w) + v001 w) + ...
__device__ __forceinline__ double mol_value(const double* __restrict__ V, int32_t n_t, int64_t n_w,
                                            int64_t ip, double tp, int64_t it, double tt, int64_t iw,
                                            double tw) {
  double value = 0.0;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int dp = (c >> 2) & 1, dt = (c >> 1) & 1, dw = c & 1;
    const double wp = dp ? tp : 1.0 - tp;
    const double wt = dt ? tt : 1.0 - tt;
    const double ww = dw ? tw : 1.0 - tw;
    const double weight = ((1.0 * wp) * wt) * ww;
    value = value + V[((ip + dp) * n_t + (it + dt)) * n_w + (iw + dw)] * weight;
  }
  return value;
}

// SerpensExosphere's density (gasProperties.py:583-601): scipy RegularGridInterpolator (linear) of the
// packed grid g = [gx[nx], gy[ny], gz[nz], values[nx][ny][nz]] at (x, y, z); NaN outside (bounds_error).
// Same brackets, weights and corner order as the molecular lookup (mol_value).
__device__ __forceinline__ double grid_value(const double* __restrict__ g, int32_t nx, int32_t ny, int32_t nz,
                                             double x, double y, double z) {
  const double* gx = g;
  const double* gy = gx + nx;
  const double* gz = gy + ny;
  const double* V = gz + nz;
  int64_t ix, iy, iz;
  double tx, ty, tz;
  if (!rgi_bracket(gx, nx, x, &ix, &tx) || !rgi_bracket(gy, ny, y, &iy, &ty) || !rgi_bracket(gz, nz, z, &iz, &tz))
    return __builtin_nan("");
  return mol_value(V, ny, nz, ix, tx, iy, ty, iz, tz);
}

__device__ __forceinline__ double grid_density(const DensityDev& m, const double* __restrict__ g, double xv,
                                               double y, double z, double bx, double by) {
  return grid_value(g, (int32_t)m.p[0], (int32_t)m.p[1], (int32_t)m.p[2], xv - bx, y - by, z);
}

}  // namespace prom
