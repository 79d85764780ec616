// Transmission-curve evaluation shared by the lookup kernels (prom_tcurve.hip: k_tc_build, k_sigma_tc; prom_tw.hip:
// k_sigma_tw).  See prom_tcurve.hip for the curves: R(o, w) = T_o(Y(o, w)), T_o(Y) = tfrac_o + sum_c F_c exp(-N_c Y),
// the sumOverChords disk sum (gasProperties.py:1241-1258) of one effective absorber.
#pragma once
#include "prom_device.h"

namespace prom {

constexpr double kTcEps = 0x1p-7;        // tail threshold of q
constexpr int kTcExpEps = -7;            // its binary exponent
constexpr double kTcSat = 40.0;          // tau above which a chord is opaque (e^-40 = 4e-18)

// q = Y N_max's binary exponent (q normal and >= 2^-7)
__device__ __forceinline__ int32_t tc_exponent(double q) {
  return (int32_t)((__builtin_bit_cast(unsigned long long, q) >> 52) & 0x7ff) - 1023;
}

// octaves [0, L) that cover q in [eps, qhi]: 0 when qhi < eps, INT32_MAX when not finite
__device__ __forceinline__ int32_t tc_octaves(double qhi) {
  if (!(qhi >= kTcEps)) return 0;
  if (!(qhi <= 1.0e300)) return 0x7fffffff;
  return tc_exponent(qhi) - kTcExpEps + 1;
}

// the octave's Chebyshev series at q (normal, inside the table): v = log2 of q's mantissa in [0, 1), Clenshaw in
// u = 2 v - 1 over the 16 coefficients c.  The coefficients come four at a time: the rare octave branch must not
// set the lookup kernels' register peak (all 16 in flight take 32 VGPRs)
__device__ __forceinline__ double tc_clenshaw(double q, const double* __restrict__ c) {
  const double m = __builtin_bit_cast(double, (__builtin_bit_cast(unsigned long long, q) & 0x000fffffffffffffull) |
                                                  0x3ff0000000000000ull);
  const double u = __builtin_fma(2.0, log2(m), -1.0);
  double b1 = 0.0, b2 = 0.0, c0 = 0.0;
#pragma unroll 1
  for (int k0 = kTcD - 4; k0 >= 0; k0 -= 4) {
    const double2 ca = *reinterpret_cast<const double2*>(c + k0), cb = *reinterpret_cast<const double2*>(c + k0 + 2);
    const double cv[4] = {ca.x, ca.y, cb.x, cb.y};
#pragma unroll
    for (int i = 3; i >= 0; --i) {
      if (k0 + i >= 1) {
        const double b0 = __builtin_fma(2.0 * u, b1, cv[i] - b2);
        b2 = b1;
        b1 = b0;
      } else {
        c0 = cv[0];
      }
    }
  }
  return __builtin_fma(u, b1, c0 - b2);
}

// The exact chord sums in chord order with ocml exp: non-finite columns (nf: the reference's order, the NaN pattern --
// tau is NaN for an infinite column where some chi_s sigma_s is not > 0, zr) or beyond a table truncated at the host's
// octave cap (F_out / F_sum weights).  Not inlined and not optimised: inlined, machine LICM hoists ocml exp's constants
// out of the lookup kernels' loops and their register allocation grows by ~10-20 VGPRs for paths that run only in
// pathological cases (k_sigma_tw; k_sigma_tc keeps them inline: there the call's saved registers cost more); the
// operations and their order are the inlined code's (tc_eval, k_sigma_tc), so the sums are bitwise the same
#ifndef PROM_TC_CS_ATTR   // (inlined instead, -DPROM_TC_CS_ATTR=__forceinline__: no scratch, 77 VGPRs, no faster: r06z)
#define PROM_TC_CS_ATTR __noinline__ __attribute__((optnone))
#endif
__device__ PROM_TC_CS_ATTR double tc_chord_sum(double Y, bool nf, bool zr, double fs,
                                                                    const int32_t* __restrict__ fl,
                                                                    const double* __restrict__ nc,
                                                                    const double* __restrict__ fout, int32_t n_pr) {
  const double inv_fs = 1.0 / fs;
  double a = 0.0;
  for (int32_t ci = 0; ci < n_pr; ++ci) {
    if (fl[ci] != 0) continue;
    const double N = nc[ci];
    double tau = N * Y;
    if (nf && zr && !__builtin_isfinite(N)) tau = __builtin_nan("");
    const double e = exp(-tau);
    a = nf ? a + fout[ci] * e : a + (fout[ci] * inv_fs) * e;
  }
  return a;
}

// T_o(Y) for a phase whose columns are finite (header h, its table rows tabo)
__device__ __forceinline__ double tc_eval(double Y, const double* __restrict__ h, const double* __restrict__ tabo,
                                          const int32_t* __restrict__ fl, const double* __restrict__ nc,
                                          const double* __restrict__ fout, int32_t n_pr, unsigned long long* evals) {
  const double q = Y * h[kTcHNmax];
  const double tf = h[kTcHTfrac];
  if (q < kTcEps) {
    double p = h[kTcHT0 + 5];
#pragma unroll
    for (int e = 4; e >= 0; --e) p = __builtin_fma(p, q, h[kTcHT0 + e]);
    return tf + p;
  }
  const int32_t nact = (int32_t)h[kTcHNact];
  if (!(q == q)) return nact > 0 ? q : tf;   // NaN cross-section: NaN wherever a chord absorbs
  const int32_t L = (int32_t)h[kTcHL];
  const int32_t j = q <= 1.0e300 ? tc_exponent(q) - kTcExpEps : 0x7fffffff;
  if (j < L) return tf + tc_clenshaw(q, tabo + (int64_t)j * kTcD);
  if ((int32_t)h[kTcHFlags] & 1) return tf;   // every chord opaque (tau >= 40)
  // beyond a truncated table: the exact sum over the phase's active chords, in chord order
  const double inv_fs = 1.0 / h[kTcHFsum];
  double a = 0.0;
#pragma unroll 1
  for (int32_t c = 0; c < n_pr; ++c)
    if (fl[c] == 0) a += (fout[c] * inv_fs) * exp(-(nc[c] * Y));
  if (evals) atomicAdd(&evals[threadIdx.x & 63], (unsigned long long)nact);
  return tf + a;
}

// fma(a, b, c) with c wave-uniform in scalar registers: one v_fma_f64 with an SGPR operand.  (Left to itself the
// compiler copies each scalar coefficient into VGPRs -- two v_mov_b32 -- and uses v_fmac: 15 VALU for the tail
// polynomial instead of 7, per point)
__device__ __forceinline__ double fma_s(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
}

// tc_eval_full with the row's header in scalar registers (h uniform): the tail polynomial by fma_s, the rest as
// tc_eval_full (the same operations in the same order: bitwise its result)
__device__ __forceinline__ double tc_eval_full_s(double Y, const double* __restrict__ h, const double* __restrict__ tabo) {
  const double q = Y * h[kTcHNmax];
  const double tf = h[kTcHTfrac];
  if (q < kTcEps) {
    double c5 = h[kTcHT0 + 5];
    asm volatile("" : "+v"(c5));   // (the leading coefficient in VGPRs: one FMA may read one scalar pair)
    double p = fma_s(c5, q, h[kTcHT0 + 4]);
#pragma unroll
    for (int e = 3; e >= 0; --e) p = fma_s(p, q, h[kTcHT0 + e]);
    return tf + p;
  }
  const int32_t nact = (int32_t)h[kTcHNact];
  if (!(q == q)) return nact > 0 ? q : tf;
  const int32_t L = (int32_t)h[kTcHL];
  const int32_t j = q <= 1.0e300 ? tc_exponent(q) - kTcExpEps : 0x7fffffff;
  if (j >= L) return tf;
  return tf + tc_clenshaw(q, tabo + (int64_t)j * kTcD);
}

// tc_eval for a phase whose table covers every q it can reach (curve header flag 4 clear: not truncated at the
// host's octave cap), so the exact per-point sum beyond the table never runs
__device__ __forceinline__ double tc_eval_full(double Y, const double* __restrict__ h, const double* __restrict__ tabo) {
  const double q = Y * h[kTcHNmax];
  const double tf = h[kTcHTfrac];
  if (q < kTcEps) {
    double p = h[kTcHT0 + 5];
#pragma unroll
    for (int e = 4; e >= 0; --e) p = __builtin_fma(p, q, h[kTcHT0 + e]);
    return tf + p;
  }
  const int32_t nact = (int32_t)h[kTcHNact];
  if (!(q == q)) return nact > 0 ? q : tf;
  const int32_t L = (int32_t)h[kTcHL];
  const int32_t j = q <= 1.0e300 ? tc_exponent(q) - kTcExpEps : 0x7fffffff;
  if (j >= L) return tf;   // (every chord opaque: the table's top is 40 N_max / N_min)
  return tf + tc_clenshaw(q, tabo + (int64_t)j * kTcD);
}

}  // namespace prom
