// Target windows of the Doppler-shifted cross-section lookups (host side, per set; k_sigma_tw in prom_tw.hip).
//
// With orbital Doppler shift every (phase o, wavelength w) looks the tables up at t = shift_o lambda_w
// (gasProperties.py:941-954: getSigmaAbs(wavelength / dopplerShift)-style shifted grids, one per phase).  A
// workgroup per 256-wavelength block needs the table nodes of all its rows' targets: the block's span plus the
// whole Doppler spread, staged again by the next block and by every other row group.  Here the target axis itself
// is cut into windows: window b is the interval [B_b, B_{b+1}) of target values; row o contributes the contiguous
// wavelengths W[b][o] <= w < W[b+1][o] with fl(shift_o lambda_w) inside it (fl(s lambda) is monotone in lambda,
// so these are ranges and the windows partition every row).  Each table node is then staged by one window only.
//
// Windows are grown greedily over candidate boundaries (the targets of a reference row, extended below and above
// by the rows with the smallest and largest factors) while every row keeps <= rowcap wavelengths, the window
// <= pmax points, and the species' slices and the wavelengths the rows read fit the workgroup's LDS (lds doubles:
// 24 bytes a node, 8 a wavelength, <= lamcap wavelengths).  Per species the slice [lo, lo + m) holds the
// bracket of every target in the window and a linear guess g(t) = clamp((int)fma(t, inv, xs), 0, m - 2) verified
// (as prom_transit_set's sigma segments) to be within one node of numpy's bracket over the window's target range;
// a window whose guess fails is shortened (bisection); a single candidate interval without one (a slice across a
// change of the table's node spacing) is searched in LDS.  kind 1: staged at pool offset pad, guessed; 2: guess into
// the global records (slice larger than the pool); 3: staged, binary search; 0: targets outside the table (numpy's
// end rules: the table's own search, the kernel's second pass).
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <thread>

#include "prom_internal.h"

namespace prom {

namespace {

struct Table {
  const std::vector<double>* X;
  int64_t bracket(double v) const {   // numpy's bracket: the largest j <= n - 2 with X[j] <= v (clamped)
    const int64_t n = (int64_t)X->size();
    int64_t j = (int64_t)(std::upper_bound(X->begin(), X->end(), v) - X->begin()) - 1;
    return j < 0 ? 0 : (j > n - 2 ? n - 2 : j);
  }
};

// the slice of targets in [tlo, thi] and its verified linear guess (prom_transit_set's make_seg, with the
// intervals' upper ends clipped to thi): false when the guess fails
bool window_slice(const std::vector<double>& X, int64_t lo, int64_t hi, double tlo, double thi, SigSeg& e) {
  const int64_t m = hi - lo + 1;
  e.lo = (int32_t)lo;
  e.m = (int32_t)m;
  e.xs = 0.0;
  e.inv = 0.0;
  if (m < 2) return false;
  const double xs = X[lo], span = X[hi] - X[lo];
  const double inv = span > 0.0 ? (double)(m - 1) / span : 0.0;
  const double b0 = -(xs * inv);
  if (!(span > 0.0) || !std::isfinite(inv) || !std::isfinite(b0)) return false;
  auto guess = [&](double v) -> int64_t {
    const double f = std::fma(v, inv, b0);   // the device's seg_guess
    return f < 0.0 ? 0 : (f >= (double)(m - 2) ? m - 2 : (int64_t)f);
  };
  for (int64_t i = lo; i < hi; ++i) {
    if (X[i] == X[i + 1]) continue;
    const double a = std::max(X[i], tlo), z = std::min(std::nextafter(X[i + 1], -INFINITY), thi);
    if (a > z) continue;
    const int64_t k = i - lo;
    const int64_t ga = guess(a), gz = guess(z);
    if (ga < k - 1 || ga > k + 1 || gz < k - 1 || gz > k + 1) return false;
  }
  e.xs = b0;
  e.inv = inv;
  return true;
}

struct Win {
  std::vector<int32_t> start;   // per row
  std::vector<SigSeg> seg;      // per species
  int32_t lw0 = 0, lw1 = 0;     // the wavelengths any row of the window reads (staged with the slices)
};

}  // namespace

bool build_target_windows(const double* wav, int64_t n_wav, const double* shift, int32_t n_rows,
                          const std::vector<const std::vector<double>*>& tabs, int32_t lds, int32_t lamcap,
                          int32_t rowcap, int64_t pmax, std::vector<SigSeg>& seg_out, std::vector<int32_t>& row_out,
                          std::vector<int32_t>& lam_out, int32_t& n_win) {
  const int NS = (int)tabs.size();
  if (n_wav < 1 || n_wav >= INT32_MAX || n_rows < 1 || NS < 1 || NS > 4 || rowcap < 1 || pmax < 1 || lds < 16 ||
      lamcap < 0)
    return false;
  // lamfit: grow windows only while their wavelengths fit the LDS beside the slices (else they are staged only where
  // they happen to fit, and read from global memory elsewhere)
  const bool lamfit = lamcap > 0 && [] { const char* e = std::getenv("PROM_TW_LAMFIT"); return e && std::atoi(e) != 0; }();
  // PROM_TW_ALIGN: the largest overhang past a multiple of 64 wavelengths per row that a window drops (0: none)
  static const int64_t align = [] { const char* e = std::getenv("PROM_TW_ALIGN"); return e ? (int64_t)std::atoi(e) : (int64_t)64; }();
  // LDS budget in doubles: 3 per staged node ({E, L} and x), one more x per species, one per staged wavelength
  auto fits = [&](int64_t nodes, int64_t lam) { return 3 * nodes + NS + lam <= lds && lam <= lamcap; };
  for (int64_t w = 0; w < n_wav; ++w)
    if (!(wav[w] > 0.0) || !std::isfinite(wav[w]) || (w > 0 && !(wav[w] > wav[w - 1]))) return false;
  for (int32_t o = 0; o < n_rows; ++o)
    if (!(shift[o] > 0.0) || !std::isfinite(shift[o])) return false;
  std::vector<Table> T(NS);
  for (int s = 0; s < NS; ++s) {
    if (tabs[s]->size() < 2) return false;
    T[s].X = tabs[s];
  }
  auto tgt = [&](int32_t o, int64_t w) -> double { return shift[o] * wav[w]; };
  // reference rows: the median factor; the smallest and largest for the ends
  std::vector<int32_t> ord(n_rows);
  for (int32_t o = 0; o < n_rows; ++o) ord[o] = o;
  std::sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return shift[a] < shift[b]; });
  const int32_t o_lo = ord.front(), o_hi = ord.back(), o_ref = ord[n_rows / 2];
  std::vector<double> C;
  C.reserve(n_wav + 1024);
  for (int64_t w = 0; w < n_wav && tgt(o_lo, w) < tgt(o_ref, 0); ++w) C.push_back(tgt(o_lo, w));
  for (int64_t w = 0; w < n_wav; ++w) C.push_back(tgt(o_ref, w));
  {
    int64_t w = 0;
    while (w < n_wav && !(tgt(o_hi, w) > tgt(o_ref, n_wav - 1))) ++w;
    for (; w < n_wav; ++w) C.push_back(tgt(o_hi, w));
  }
  C.erase(std::unique(C.begin(), C.end()), C.end());
  const int64_t K = (int64_t)C.size();
  double tmin_all = INFINITY, tmax_all = -INFINITY;
  for (int32_t o = 0; o < n_rows; ++o) {
    tmin_all = std::min(tmin_all, tgt(o, 0));
    tmax_all = std::max(tmax_all, tgt(o, n_wav - 1));
  }
  // boundary j = 0 .. K + 1: -inf, C[0 .. K), +inf; W_o(j) = #{w : t_o(w) < B_j}
  auto bnd = [&](int64_t j) -> double { return j == 0 ? -INFINITY : (j > K ? INFINITY : C[j - 1]); };
  auto count_below = [&](int32_t o, double v) -> int64_t {
    int64_t a = 0, b = n_wav;   // first w with t_o(w) >= v
    while (a < b) {
      const int64_t mid = (a + b) >> 1;
      if (tgt(o, mid) < v) a = mid + 1; else b = mid;
    }
    return a;
  };
  // the windows' target range: [B_j, B_e) clipped to the actual targets
  auto t_lo = [&](int64_t j) { return std::max(bnd(j), tmin_all); };
  auto t_hi = [&](int64_t e) { return e > K ? tmax_all : std::min(std::nextafter(bnd(e), -INFINITY), tmax_all); };
  // greedy over candidate boundaries [j0, j1): one host thread per chunk (windows end at chunk edges)
  auto greedy = [&](int64_t j0, int64_t j1, std::vector<Win>& out) {
    std::vector<int64_t> Pa(n_rows), Pb(n_rows), Pt(n_rows);
    for (int32_t o = 0; o < n_rows; ++o) Pa[o] = j0 == 0 ? 0 : count_below(o, bnd(j0));
    std::vector<int64_t> hs(NS);
    int64_t j = j0;
    while (j < j1) {
      // window [B_j, B_e), e = j + 1 always; grown while the caps hold
      const double tlo = t_lo(j);
      std::vector<int64_t> blo(NS);
      for (int s = 0; s < NS; ++s) hs[s] = blo[s] = T[s].bracket(tlo);
      Pb = Pa;
      int64_t e = j;
      while (e < j1) {
        const int64_t e2 = e + 1;
        const double bv = bnd(e2);
        int64_t tot = 0, mx = 0, la = INT64_MAX, lz = 0;
        for (int32_t o = 0; o < n_rows; ++o) {
          int64_t p = Pb[o];
          while (p < n_wav && tgt(o, p) < bv) ++p;
          Pt[o] = p;
          tot += p - Pa[o];
          mx = std::max(mx, p - Pa[o]);
          if (p > Pa[o]) {
            la = std::min(la, Pa[o]);
            lz = std::max(lz, p);
          }
        }
        const int64_t lam = lz > la ? lz - la : 0;
        const double thi = t_hi(e2);
        int64_t nodes = 0;
        for (int s = 0; s < NS; ++s) {
          const std::vector<double>& X = *T[s].X;
          int64_t h = hs[s];
          while (h < (int64_t)X.size() - 2 && X[h + 1] <= thi) ++h;
          nodes += h + 1 - blo[s] + 1;
        }
        if (e2 > j + 1 && (mx > rowcap || tot > pmax || !fits(nodes, lamfit ? lam : 0))) break;
        e = e2;
        Pb.swap(Pt);
        for (int s = 0; s < NS; ++s) {
          const std::vector<double>& X = *T[s].X;
          while (hs[s] < (int64_t)X.size() - 2 && X[hs[s] + 1] <= thi) ++hs[s];
        }
      }
      // lane alignment: a row's wavelengths are computed 64 at a time, so a window whose longest row ends a few
      // wavelengths past a multiple of 64 (C3: ~200 = 3 full chunks + 8) spends a nearly empty fourth chunk on every
      // row.  When the overhang is at most `align` wavelengths, end the window where the longest row holds exactly
      // that multiple (the next window starts there); the counts of a window's rows differ by the Doppler spread only
      if (align > 0 && e > j + 1) {
        int64_t mxe = 0;
        for (int32_t o = 0; o < n_rows; ++o) mxe = std::max(mxe, Pb[o] - Pa[o]);
        const int64_t cap = mxe / 64 * 64;
        if (cap >= 64 && mxe > cap && mxe - cap <= align) {
          auto mx_at = [&](int64_t ee) {
            int64_t m = 0;
            for (int32_t o = 0; o < n_rows; ++o) m = std::max(m, (ee > K ? n_wav : count_below(o, bnd(ee))) - Pa[o]);
            return m;
          };
          int64_t g = j + 1, b = e;   // the largest e' in [j + 1, e) with mx_at(e') <= cap (mx_at(e) > cap)
          if (mx_at(g) <= cap) {
            while (b - g > 1) {
              const int64_t mid = (g + b) >> 1;
              if (mx_at(mid) <= cap) g = mid; else b = mid;
            }
            e = g;
            for (int32_t o = 0; o < n_rows; ++o) Pb[o] = e > K ? n_wav : count_below(o, bnd(e));
          }
        }
      }
      // per species slice and guess; shorten the window while some in-range species' guess fails
      Win wn;
      wn.seg.assign(NS, SigSeg{0, 0, 0, 0, 0.0, 0.0});
      auto try_e = [&](int64_t ee, bool commit) -> bool {
        const double a = t_lo(j), z = t_hi(ee);
        bool ok = true;
        for (int s = 0; s < NS; ++s) {
          const std::vector<double>& X = *T[s].X;
          SigSeg sg{0, 0, 0, 0, 0.0, 0.0};
          const bool inr = a >= X.front() && z < X.back() && a <= z;
          if (inr) {
            const int64_t lo = T[s].bracket(a), hi = T[s].bracket(z) + 1;
            if (window_slice(X, lo, hi, a, z, sg)) sg.kind = 2;
            else {
              sg.kind = 4;   // (in range, no guess: staged and searched when it fits the pool)
              ok = false;
            }
          }
          if (commit) wn.seg[s] = sg;
        }
        return ok;
      };
      if (!try_e(e, false) && e > j + 1) {
        int64_t g = j + 1, b = e;   // try_e(g) assumed; find the largest valid e' in [j + 1, e)
        if (try_e(g, false)) {
          while (b - g > 1) {
            const int64_t mid = (g + b) >> 1;
            if (try_e(mid, false)) g = mid; else b = mid;
          }
        }
        e = g;
        for (int32_t o = 0; o < n_rows; ++o) Pb[o] = count_below(o, bnd(e));
        if (e > K) for (int32_t o = 0; o < n_rows; ++o) Pb[o] = n_wav;
      }
      try_e(e, true);
      // the wavelengths the window's rows read
      int64_t la = INT64_MAX, lz = 0;
      for (int32_t o = 0; o < n_rows; ++o)
        if (Pb[o] > Pa[o]) {
          la = std::min(la, Pa[o]);
          lz = std::max(lz, Pb[o]);
        }
      const int64_t lam = lz > la ? lz - la : 0;
      wn.lw0 = lz > la ? (int32_t)la : 0;
      int64_t need = 0;   // (the slices come first; the wavelengths are staged only in what LDS they leave)
      for (int s = 0; s < NS; ++s)
        if (wn.seg[s].kind == 2 || wn.seg[s].kind == 4) need += wn.seg[s].m;
      wn.lw1 = fits(need, lam) ? (int32_t)(wn.lw0 + lam) : wn.lw0;   // (lw1 = lw0: global loads)
      const int64_t pool = (lds - NS - (wn.lw1 - wn.lw0)) / 3;
      // pool offsets for the guessed slices, species order, while they fit
      int32_t off = 0;
      for (int s = 0; s < NS; ++s) {
        SigSeg& sg = wn.seg[s];
        if ((sg.kind == 2 || sg.kind == 4) && off + sg.m <= pool) {
          sg.kind = sg.kind == 2 ? 1 : 3;
          sg.pad = off;
          off += sg.m;
        } else if (sg.kind == 4) {
          sg.kind = 0;
        }
      }
      int64_t tot = 0;
      for (int32_t o = 0; o < n_rows; ++o) tot += Pb[o] - Pa[o];
      if (tot > 0) {
        wn.start.resize(n_rows);
        for (int32_t o = 0; o < n_rows; ++o) wn.start[o] = (int32_t)Pa[o];
        out.push_back(std::move(wn));
      }
      Pa = Pb;
      j = e;
    }
  };
  const int64_t nb = K + 1;   // candidate intervals
  const int64_t n_thr = std::max<int64_t>(1, std::min<int64_t>(8, nb / 65536));
  std::vector<std::vector<Win>> parts(n_thr);
  {
    std::vector<std::thread> pool_t;
    for (int64_t t = 1; t < n_thr; ++t)
      pool_t.emplace_back(greedy, nb * t / n_thr, nb * (t + 1) / n_thr, std::ref(parts[t]));
    greedy(0, nb / n_thr, parts[0]);
    for (auto& th : pool_t) th.join();
  }
  seg_out.clear();
  row_out.clear();
  lam_out.clear();
  n_win = 0;
  for (auto& p : parts)
    for (auto& wn : p) {
      row_out.insert(row_out.end(), wn.start.begin(), wn.start.end());
      seg_out.insert(seg_out.end(), wn.seg.begin(), wn.seg.end());
      lam_out.push_back(wn.lw0);
      lam_out.push_back(wn.lw1);
      ++n_win;
    }
  for (int32_t o = 0; o < n_rows; ++o) row_out.push_back((int32_t)n_wav);
  return n_win > 0;
}

}  // namespace prom
