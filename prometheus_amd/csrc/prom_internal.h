// Internal declarations shared by the C-ABI layer (prom_api.hip) and the kernels (prom_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/prom_hip.h"

namespace prom {

struct Error : std::runtime_error {
  int32_t code;
  Error(int32_t c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define PROM_HIP(expr)                                                                      \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      throw ::prom::Error(PROM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));   \
  } while (0)

#define PROM_REQUIRE(cond, msg)                                     \
  do {                                                              \
    if (!(cond)) throw ::prom::Error(PROM_E_ARG, std::string(msg)); \
  } while (0)

// Grow-only device buffer owned by a context.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      release();
      p = o.p; cap = o.cap;
      o.p = nullptr; o.cap = 0;
    }
    return *this;
  }
  ~DevBuf() { release(); }
  void ensure(size_t bytes) {
    if (bytes <= cap) return;
    release();
    if (bytes == 0) return;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
      p = nullptr;
      throw Error(PROM_E_NOMEM, "hipMalloc(" + std::to_string(bytes) + " B): " + hipGetErrorString(e));
    }
    cap = bytes;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

constexpr int kCnt = 8;   // int32 counters per phase in TransitDev::counts
constexpr int kMolMirrorMax = 8192;   // chords per phase for k_mol_list's mirror merging (32 KB of LDS)
constexpr int kMolListPad = 4;   // valid zero-weight entries after each phase's molecular sample list (k_mol_list)

// Windowed integration (prom_kernels.hip, "windowed integration"): per-phase ordering limit, the
// size of the per-phase threshold -> record-index tables, and the number of tail moments for S
// atomic species.
constexpr int kWinMax = 4096;
constexpr int kEnvN = 2048;
constexpr int kWinMaxSpecies = 4;
// (prom_kernels.hip Monos / TailDeg: degree 7 for one effective species, 3 otherwise)
inline int n_tail_moments(int S) { return S == 1 ? 8 : (S + 1) * (S + 2) * (S + 3) / 6; }

// Doppler cross-section rows: table nodes a resampling workgroup stages in LDS per species (prom_api.hip
// sigma segments; larger slices gather from the global table).
#ifndef PROM_SIG_SEG
#define PROM_SIG_SEG 416   // (LDS slice cap: 416 nodes keep a 3-species k_sigma_tc workgroup at 31 KB; r04o sweep)
#endif
constexpr int kSigSeg = PROM_SIG_SEG;
// k_sigma_tc's LDS slice cap by the number of staged species (24 bytes a node: ~24-31 KB a workgroup).  One species
// takes slices up to 1,024 nodes: a block's targets over every phase's Doppler shift (C4x10: ~860 nodes for 256
// wavelengths at 0.001 A under a 0.6 A Doppler spread) stay in LDS instead of the global-record front path.  Host
// segments mark slices within the cap SigSeg kind & 64.
constexpr int tc_slice_cap(int nsig) { return nsig <= 1 ? 1024 : (nsig == 2 ? 640 : kSigSeg); }
#ifndef PROM_TW_LDSD
#define PROM_TW_LDSD 2816   // (build macro for A/B builds; 7 workgroups per CU fit up to 2,861 -- the SGPRs allow 7 waves)
#endif
// k_sigma_tw: LDS doubles per workgroup (22 KB): staged nodes (3 each) + wavelengths.  2,816 against 2,560: the C3
// windows stage their wavelengths in 1,830 of 1,859 windows instead of 513 of 1,863, C3 0.0371 -> 0.0364-0.0367 ms,
// C4x10 0.0570-0.0577 -> 0.0559-0.0570 ms per step on one box (profiles/r06_tw_ab_sessions.txt, r06q2)
constexpr int kTwLds = PROM_TW_LDSD;
constexpr int kTwLamCap = 1024;   // ... wavelengths staged per window at most
constexpr int kSigBlockW = 256;   // wavelengths per resampling workgroup (== kBlock)
#ifndef PROM_SIG_ROWS
#define PROM_SIG_ROWS 8
#endif
constexpr int kSigRowChunk = PROM_SIG_ROWS;   // rows per resampling workgroup (4, 8 or 16)

// Stellar-spectrum path: star-table nodes a tau workgroup stages in LDS (prom_api.hip rm_slices).
constexpr int kRmStarMax = 1024;

// Device-side view of one density model (the prom_density_model scalars).
struct DensityDev {
  int32_t kind;
  int32_t pad;      // POWERLAW: q + 1 when q is an integer in [0, 64] (repeated squaring), else 0
  double p[8];
};

// Per-scenario view for the streaming column kernel (layout shared with prom_kernels.hip's ScDev).
struct ScDevHost {
  DensityDev m;
  const double* tab;
};

// Device-side descriptor of one absorbing constituent inside the transit problem.
struct TermDev {
  int32_t scenario;     // index of its density scenario
  int32_t is_molecule;
  int32_t slot;         // atomic: index into N / sigma arrays;  molecular: molecular slot
  int32_t table;        // table id
  double chi;
};

// Per atomic slot of a transit problem: its table and its scenario's per-phase Doppler factors.
struct SigTabDev {
  const double* x;
  const double* y;
  int64_t n;
  double offset;
  const double* shift;   // [n_orb]
  const int32_t* dir;    // [n_dir + 1] bucket directory of x (AtomTable::dir)
  int32_t n_dir;
  int32_t pad;
  double dir_x0, dir_inv_h;
  double ncoef;          // c_s: column normalisation of the windowed integration (n = c_s N <= 1)
  double nscale;         // 1 / c_s (0 when c_s == 0)
  double chi;            // the constituent's mixing ratio (species merging: Y = sum_s chi_s sigma_s)
  double xfirst, xlast;  // x[0], x[n - 1] (range test without a dependent load)
  const double4* rec;    // [n] {x_i, y_i, slope_i = (y_{i+1} - y_i) / (x_{i+1} - x_i), 0} (AtomTable::rec)
};

// one destination of prom_transit_set's staged upload: bytes at src_off of the staging buffer -> dst
struct ScatterDesc {
  void* dst;
  int64_t src_off;
  int64_t bytes;
};

// Per 256-wavelength block and atomic slot of a Doppler-row problem (prom_api.hip sigma segments): the
// table nodes [lo, lo + m) every row's targets fall between, and, for kind > 0, a linear bracket guess
// g(t) = clamp((int)fma(t, inv, xs), 0, m - 2) (xs holds -x_lo inv) that the host verified to be within one node of numpy's
// bracket for every target in the slice.  kind & 3: 0 no guess (general lookup); 1 the slice fits in LDS;
// 2 too large for LDS, the guess indexes the global records.  kind & 4 (k_seg_exact, at prom_transit_set):
// the guess IS numpy's bracket for every target of the block's rows (one record read, no compares).  kind & 64: a
// guess and m <= tc_slice_cap(species of the problem) (k_sigma_tc stages the slice in LDS).
struct SigSeg {
  int32_t lo, m, kind, pad;
  double xs, inv;
};

// Per molecular slot of a transit problem.
// Per 32-chord group of one phase (k_columns8, transmission-curve path): the order-independent phase sums
// k_tc_build needs before its node sums (max / min of the active finite columns, chord counts by class)
struct TcPart {
  double nmax, nmin;
  int32_t nact, ntr, nbl, nnf;
};

struct MolSlotDev {
  const double* P;       // [n_p] dyn cm^-2
  const double* T;       // [n_t]
  const double* W;       // [n_w] cm
  const double* V;       // [n_p][n_t][n_w] log10(xsec + offset)
  int32_t n_p, n_t;
  int64_t n_w;
  double offset;
  double fill;           // log10(offset): RegularGridInterpolator fill value
  double temp;           // the scenario's T (lookup temperature; P = n k_B T)
  double chi;
  double k_B;
  const double* shift;   // [n_orb] Doppler factors of its scenario
  int32_t scenario;
  int32_t pad;
  const double2* G;      // [max(n_p - 1, 1)][n_w - 1][2] bilinear records of V lerped to the slot's T (k_mol_gt, per set)
};

// Terms and scenarios of small problems passed by value to the column kernel.
struct ColArgs {
  TermDev t[8];
  ScDevHost sc[4];
};

// Tables of up to kWinMaxSpecies atomic slots passed by value (kernel arguments: no dependent load).
struct SigTabs4 {
  SigTabDev t[4];
};

// The transmission-curve path (prom_tcurve.hip): per phase a header of kTcHdr doubles and kTcD Chebyshev
// coefficients per octave of q = Y N_max.
constexpr int kTcHdr = 16;
constexpr int kTcD = 16;
enum : int { kTcHNmax = 0, kTcHTfrac = 1, kTcHFsum = 2, kTcHT0 = 3 /* .. 8: tail coefficients t_0 .. t_5 */,
             kTcHL = 9, kTcHFlags = 10 /* 1: opaque above the table, 2: non-finite columns, 4: truncated at the octave cap */, kTcHNact = 11 };
constexpr int kTcMaxOctaves = 64;
constexpr int kTcChain = 4;                          // octaves per table exp (k_tc_build)
constexpr int kTcPartMax = 16;                       // chord parts per (phase, chain)
constexpr int kTcPartVals = (kTcChain + 1) * kTcD;   // doubles per part: node sums per octave, then the moments

struct TcArgs {
  const double* hdr;         // [n_orb][kTcHdr]
  const double* tab;         // [n_orb][lg][kTcD]
  const int32_t* flags;      // [n_orb][n_pr] chord flags (0 active)
  const double* ncol;        // [n_orb][n_pr] the effective absorber's columns
  const double* fout;        // [n_pr]
  double* R;                 // [n_orb][n_wav]
  unsigned long long* evals; // [64] exp-evaluation counters (stats runs) or null
  int32_t lg, n_pr;
};

struct AtomTable {
  bool live = false;     // slot in use (prom_table_free releases it for reuse)
  DevBuf x, y;
  int64_t n = 0;
  double offset = 0.0;
  double ymax = 0.0;     // max of y (log10 sigma): sigma_max = 10^ymax - offset
  // bucket directory for O(1) bracketing: dir[j] = #{i : x[i] <= x0 + j h}, j = 0 .. n_dir,
  // h = (x[n-1] - x0) / n_dir (prom_api.hip build_directory)
  DevBuf dir;
  DevBuf rec;               // [n] double4 {x_i, 10^y_i, ln10 slope_i, x_{i+1}} (k_table_recs)
  double amax = 0.0;        // max over intervals of |ln10 slope_i| (x_{i+1} - x_i) (NaN: non-finite y)
  std::vector<double> hx;   // host copy of x (stellar-spectrum slice bounds)
  int32_t n_dir = 0;
  double dir_x0 = 0.0, dir_inv_h = 0.0;
  uint64_t gen = 0;         // upload number within the context (ids are reused, generations are not)
};

struct MolTable {
  bool live = false;
  DevBuf P, T, W, V;
  int32_t n_p = 0, n_t = 0;
  int64_t n_w = 0;
  double offset = 0.0;
  double vmax = 0.0;
};

// Work and output buffers of one run.  Fast-path problems rotate consecutive runs over `depth` slots
// and as many streams (PROM_PIPELINE, default 4), so that a run's column / ordering kernels overlap
// the previous runs' tau kernels; every run is complete and independent.
constexpr int kMaxSlots = 8;
struct RunSlot {
  DevBuf ncol;                              // [n_atoms][n_orb][n_pr]
  DevBuf flags;                             // [n_orb][n_pr] int32: 0 active, 1 transparent, 2 blocked
  DevBuf recs;                              // [n_orb][n_pr][1 + n_atoms] chord-order records {F/Fsum, N_s}
  DevBuf act_ip;                            // [n_orb][n_pr] int32 chord positions of the records
  DevBuf counts;                            // [n_orb][kCnt] int32 (k_order / k_chords)
  DevBuf tsum;                              // [n_orb] transparent flux sum / F_out sum
  DevBuf fsum;                              // [n_orb] F_out sum
  DevBuf mrecs;                             // sorted (+ merged) records [n_orb][n_pr][1 + n_atoms]
  DevBuf wenv;                              // [n_orb][2][kEnvN] int32 threshold -> record tables
  DevBuf wmom;                              // [n_orb][n_pr + 1][K] suffix tail moments
  DevBuf evals;                             // [64] uint64 exp-evaluation counters (stats runs)
  DevBuf sig;                               // resampled sigma_s(shift lambda_w) [sig rows][n_atoms or 1][n_wav]
  // the generic column path's and the molecular path's per-run buffers (per slot: pipelined runs)
  DevBuf ntot;                              // [n_sc][n_orb][n_pr][n_x]
  DevBuf molcol;                            // [n_mol][n_orb][n_pr] sum_x n_abs*dx (for the bound)
  DevBuf mol_smp;                           // [n_mol][n_orb][n_pr][n_x] double4 {P weight, n_abs = n chi, P bracket,
                                            //     0} of the in-table samples, compacted to the front of each chord
  DevBuf mol_nin;                           // [n_mol][n_orb][n_pr] int32 their count
  DevBuf mol_lst;                           // [n_orb][n_pr (n_mol n_x + 1) + kMolListPad] double4: each phase's records' in-table
                                            //     samples, one flat list (k_mol_list)
  DevBuf mol_rend;                          // [n_orb][n_pr] int32: end of each record's samples in the list
                                            //     (one row, or one per phase with orbital Doppler shift)
  DevBuf zfl;                               // merged species: some chi_s sigma_s not > 0 [sig rows][n_wav] uint8
  DevBuf tq;                                // resampled path: Q ranges of the two halves of each 128-lambda
                                            //     tile [sig rows][n_tiles] float4 (k_columns8)
  DevBuf trec;                              // ... each tile's tau window and flags {h, t, flags, 0} per phase
                                            //     [n_orb][n_tiles] int4 (k_order)
  DevBuf hlist;                             // ... heavy entries {half tile, h, t, flags | phase << 8}: small
                                            //     list [n_orb * 2 n_tiles], then big list [n_orb * 2 n_tiles] int4
  DevBuf hcnt;                              // ... their counts (int32 small, big; zeroed by k_columns8)
  DevBuf R;                                 // [n_orb][n_wav]
  DevBuf tc_hdr;                            // transmission curves: [n_orb][kTcHdr] (k_tc_build)
  DevBuf tc_tab;                            // ... [n_orb][tc_lg][kTcD] Chebyshev coefficients (k_tc_build)
  DevBuf tc_part;                           // ... per (phase, chain, part) node sums and moments
  DevBuf tc_cnt;                            // ... per (phase, chain) arrival counters (zero between runs)
  DevBuf tc_pp;                             // ... [n_orb][n_pr / 32] TcPart from k_columns8 (n_pr % 32 == 0)
  // second stream of the slot and its fork / join events (the Doppler sigma rows run beside the column
  // and ordering kernels); set per run by prom_transit_run, null: one stream
  hipStream_t aux = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // one stream, Doppler sigma rows queued after k_order instead of before k_columns8 (set per run by
  // prom_transit_run on alternate slots of a pipelined problem: staggers the slots' kernel order)
  bool sig_late = false;
};

// Everything the transit kernels need, as device pointers.
struct TransitDev {
  int64_t n_wav = 0;
  int32_t n_pr = 0, n_orb = 0, n_x = 0, n_sc = 0, n_moons = 0;
  int32_t n_atoms = 0, n_mol = 0, n_terms = 0;
  double delta_x = 0.0, planet_R = 0.0, cull_tau = 0.0;
  bool ready = false;
  bool ran = false;
  std::vector<TermDev> terms;               // host copy, scenario/constituent order
  std::vector<DensityDev> dens;             // host copy
  std::vector<double> atom_sigma_max;       // per atomic slot
  std::vector<double> mol_T;                // per molecular slot
  // device buffers
  DevBuf wav, cy, cz, cfout, x, planet_y, moon_y, moon_R;
  DevBuf body_x, body_y, shift;             // [n_sc][n_orb]
  DevBuf dens_dev;                          // [n_sc] DensityDev
  DevBuf scdev;                             // [n_sc] ScDev (density + tabulated pointer)
  DevBuf terms_dev;                         // [n_terms] TermDev
  DevBuf tab;                               // tabulated densities, raw host order, concatenated
  DevBuf sigma;                             // [n_atoms][n_orb][n_wav]
  DevBuf sigma_max_dev;                     // [n_atoms]
  DevBuf sigtab;                            // [n_atoms] SigTabDev
  SigTabs4 sigtab_v{};                      // the first (up to) 4 slots, for kernel arguments
  ColArgs colargs{};                        // terms / scenarios by value (n_terms <= 8, n_sc <= 4)
  int32_t exp_mode = 1;                     // 1: table-driven exp in k_tau, 0: ocml exp
  bool merge = true;                        // merge chords with equal (2^-40) column densities
  bool window = true;                       // windowed integration with tail moments
  bool uniform_shift = false;               // every atomic species' Doppler factor equal at all phases
  bool count_evals = false;
  bool plan = true;                         // planned tau integration where it applies (PROM_TAU_PLAN=0: off)
  // Species merging (PROM_SPECIES_MERGE=0: off): when every atomic constituent belongs to one density
  // scenario, tau_c(lambda) = N_c Y(lambda) with N_c = dx sum_x n and Y = sum_s chi_s sigma_s, so the
  // no-Doppler fast path integrates one effective absorber: one column per chord, one resampled
  // cross-section per wavelength, scalar windows and 4 tail moments.
  bool species_merge_ok = false;
  ColArgs colargs_m{};                      // the single chi = 1 term
  SigTabs4 sigtab_m{};                      // t[0]: the effective absorber's normalisation (ncoef, nscale)
  DevBuf sigma_max_m;                       // [1] sum_s chi_s sigma_max_s
  // upper bounds of the normalised Q = sum_s sigma_s / c_s over every wavelength and phase (per species /
  // merged): k_order's always-tail threshold btail = tail epsilon / Q bound
  double qbound_v = 0.0, qbound_m = 0.0;
  int32_t taup_resident = 0;                // k_tau_p wavefronts resident at once (set at the first run)
  // timed runs: k_tau_p stamps each workgroup's first and last device-clock tick into ts_out[2 b],
  // ts_out[2 b + 1] when it has at most ts_cap workgroups; ts_blocks reports the count (0: no stamps)
  unsigned long long* ts_out = nullptr;
  int32_t ts_cap = 0;
  int32_t ts_blocks = 0;
  // prom_transit_kernel_ms: start/stop events per kernel id (null: not profiling) and the ids launched
  hipEvent_t* kprof = nullptr;
  uint32_t kprof_mask = 0;
  DevBuf molslot;                           // [n_mol] MolSlotDev
  DevBuf mirror;                            // [n_pr] int32: each chord's mirror image (z -> -z) or -1 (host-paired)
  int64_t n_mirror = 0;                     // (mirror pairs; 0: none, or PROM_MOL_MIRROR=0)
  bool mol_stage = true;                    // k_tau_mol's LDS stage of G (PROM_MOL_STAGE=0: global reads, validation)
  std::vector<int32_t> mirror_h;            // (host image of mirror)
  DevBuf sig_seg4;                          // [n_blk][n_atoms][4] per-wavefront SigSeg of blocks without a guess (kind & 8),
                                            // then the bucket directories' SigSeg (kind & 32)
  int64_t sig_noguess = 0;                  // (block, species) pairs without a guess or a directory (host count)
  DevBuf sig_dir;                           // the bucket directories (bracket at each bucket's start, slice-relative)
  DevBuf rm_fout;                           // stellar spectrum: [n_wav] unocculted flux sum_c F(c, w) (k_rm_fout, per set)
  DevBuf rm_ftab;                           // ... [n_pr][n_wav] every chord's flux F(c, w) (k_rm_fout, per set), when it
  bool rm_ftab_ok = false;                  //     fits PROM_RM_FTAB_MB and a quarter of the free device memory
  DevBuf mol_g;                             // every slot's MolSlotDev::G
  std::vector<MolSlotDev> mslots;           // host copy
  std::vector<int64_t> tab_off;             // per scenario offset into `tab` (-1: none)
  int32_t star_table_id = -1;               // prom_transit_problem.star_table (invalidation on free)
  // stellar spectrum (prom_transit_problem.has_star)
  bool star = false;
  bool star_uniform = false;                // every chord's stellar shift equal (no rotation)
  SigTabDev star_tab{};                     // the F_star table (x, log10 F, offset 0; shift unused)
  DevBuf crho, cclv, cshift;                // [n_pr]
  DevBuf rm_slices;                         // [n_wav tiles of kBlock][3] {lo, m, half}: LDS slice
  // orbital Doppler shift: per 256-wavelength block and atomic slot, the table nodes {lo, m} every
  // phase's shifted targets fall between (m = 0: more than kSigSeg, the block gathers per target)
  DevBuf sig_seg;                           // [n_wav blocks][n_atoms] SigSeg
  DevBuf sig_fb;                            // blocks with an oversize slice (m = 0 for some species)
  int32_t n_sig_fb = 0;
  DevBuf sig_fb_tc;                         // the same for k_sigma_tc's caps (tc_slice_cap: SigSeg kind & 64)
  int32_t n_sig_fb_tc = 0;
  bool sig_seg_ok = false;
  // target windows (prom_window.hip, k_sigma_tw): per window and atomic slot a SigSeg (kind 1: pad = pool offset),
  // per window boundary and row the first wavelength; built with the sigma segments (same inputs, same reuse)
  DevBuf tw_seg;                            // [n_tw][n_atoms] SigSeg
  DevBuf tw_row;                            // [n_tw + 1][n_orb] int32
  DevBuf tw_lam;                            // [n_tw][2] int32: the wavelengths [lw0, lw1) staged per window (lw1 = lw0: none)
  int32_t n_tw = 0;
  bool tw_ok = false;
  bool tw_new = false;                      // (built by this set: the exact marks are still to come)
  // polynomial sigma rows (k_sigma_poly): degree D of the e^a Taylor polynomial for this problem's tables
  // (0: the exp10 path, k_sigma_rows; PROM_SIG_POLY=0 forces it)
  int32_t sig_deg = 0;
  DevBuf sig_flags;                         // [n_wav blocks][n_atoms] int32 (k_seg_exact)
  // inputs the sigma segments were built from (wavelengths, per-slot table generation and Doppler factors):
  // a later problem with the same ones reuses sig_seg / sig_fb instead of rebuilding them
  std::vector<double> seg_key_wav, seg_key_sh;
  std::vector<uint64_t> seg_key_gen;
  bool seg_key_valid = false;
  // transmission-curve path (prom_tcurve.hip; PROM_TCURVE=0: off): set-time switch, the octave cap of the
  // tables and the bound of Y (the effective absorber's sigma maximum) that sets each phase's table extent
  bool tcurve = true;
  int32_t tc_lg = 1;
  DevBuf tc_const;                          // k_tc_build constants: Chebyshev matrix [kTcD][kTcD], node factors [kTcD]
  int32_t tc_parts = 1;
  double tc_fsum = 0.0;                     // sum of the chords' F_out (every phase's disk sum; per set)
  bool tc_pp_ok = false;                    // this run's k_columns8 wrote the curves' phase partials (launch_transit)                     // chord parts per (phase, chain) of k_tc_build
  double tc_ybound = 0.0;
  RunSlot slot[kMaxSlots];
  // PROM_GRAPH=1: a fast-path run is one hipGraph per slot, captured at the slot's first untimed run
  // and replayed (one host call instead of three launches; slower on ROCm 7.2, so off by default)
  hipGraphExec_t gexec[kMaxSlots] = {};
  bool graphs = false;
  int8_t env_fork = -1;       // PROM_SIGMA_FORK at prom_transit_set (-1: unset)
  bool env_stagger = false;   // PROM_SIG_STAGGER at prom_transit_set
  int depth = 1;                            // slots in use: fast path = pipeline depth, else 1
  int cu_count = 0;                         // the context device's compute units (launch_tau_mol; 0: not queried yet)
  int last = 0;                             // slot of the most recent run
};

}  // namespace prom

struct prom_ctx {
  int32_t device = 0;
  hipStream_t stream = nullptr;  // slot-0 stream (and the stream of every non-run call)
  hipStream_t streams[prom::kMaxSlots] = {};   // streams[0] == stream
  int pipeline = 4;              // PROM_PIPELINE (1 .. kMaxSlots)
  hipEvent_t ev[8] = {};
  std::string err;
  std::vector<prom::AtomTable> tables;
  std::vector<prom::MolTable> mtables;
  prom::TransitDev tr;
  prom::DevBuf scratch[6];
  bool timing = false;
  std::vector<hipEvent_t> tev;   // pool, 4 per timed run
  std::vector<prom::DevBuf> tsbuf;     // pool, one per timed run: tau-kernel workgroup clock stamps
  std::vector<int32_t> ts_blocks;      // per timed run: stamped workgroups (0: none)
  int32_t timed_runs = 0;
  int32_t timing_stride = 1;     // prom_timing_stride: events on every k-th run of a timing window
  int64_t window_runs = 0;       // runs since prom_timing_begin
  // prom_transit_result: pinned staging for the D2H of R, copied out by host threads chunk by chunk
  void* pin = nullptr;
  size_t pin_cap = 0;
  std::vector<hipEvent_t> pin_ev;
  hipEvent_t fork_ev[prom::kMaxSlots] = {}, join_ev[prom::kMaxSlots] = {};
  uint64_t table_gen = 0;        // uploads so far (AtomTable::gen)
  // prom_transit_set: its small inputs staged in page-locked memory, copied in one DMA and scattered
  void* upin = nullptr;
  size_t upin_cap = 0;
  prom::DevBuf ustage;
};

namespace prom {

// ---- kernel launchers (prom_kernels.hip) ----
void launch_table_lookup(hipStream_t s, const double* x, const double* y, int64_t n, double offset,
                         const double* targets, int64_t nt, double* out);
void launch_voigt(hipStream_t s, const double* x, int64_t n, const double* lw, const double* lg,
                  const double* lc, int32_t nl, double sigma_v, double c_light, double offset,
                  int log_table, double* out);
void launch_density(hipStream_t s, const DensityDev& m, const double* x, int32_t n_x, const double* y,
                    const double* z, const double* bx, const double* by, int64_t n_chords, double* out);
void launch_molecular_sigma(hipStream_t s, const MolTable& t, int64_t n_chords, int32_t n_x,
                            const double* P, double T, int64_t n_wav, const double* wav, double* out);
// ev (may be null): {start, columns+ordering done, tau start, tau done}; stage_events false: only the
// tau pair (the fast path carries them on the tau kernel's dispatch packet)
void launch_transit(hipStream_t s, TransitDev& tr, RunSlot& rs, const std::vector<AtomTable>& tables,
                    const std::vector<MolTable>& mtables, hipEvent_t* ev, int* variant, bool stage_events);
// orbital Doppler shift: the per-phase cross-section rows, Y or sigma_s, and the Q ranges (prom_sigma.hip)
void launch_sigma_rows(hipStream_t s, int32_t nsig, const SigTabs4& tabv, const double* wav, int64_t n_wav,
                       int32_t n_rows, const SigSeg* seg, const int32_t* fb, int32_t n_fb, double* sig, float4* tq,
                       int32_t merge_sp, double nscale_m, uint8_t* zfl, hipEvent_t ev_start, hipEvent_t ev_stop);
// the same rows with e^a polynomials over the tables' {x, 10^y, ln10 slope, x_next} records (prom_sigma.hip)
void launch_sigma_poly(hipStream_t s, int32_t nsig, int32_t deg, const SigTabs4& tabv, const double* wav, int64_t n_wav,
                       int32_t n_rows, const SigSeg* seg, const int32_t* fb, int32_t n_fb, double* sig, float4* tq,
                       int32_t merge_sp, double nscale_m, uint8_t* zfl, hipEvent_t ev_start, hipEvent_t ev_stop);
// prom_transit_set: mark the sigma segments whose guess is numpy's bracket for every target (kind |= 4)
void launch_seg_exact(hipStream_t s, int32_t nsig, const SigTabs4& tabv, const double* wav, int64_t n_wav,
                      int32_t n_rows, SigSeg* seg, int32_t* flags);
// the transmission-curve path after the column kernel: k_tc_build, k_sigma_tc (prom_tcurve.hip);
// the event pairs (may be null) ride on the two kernels' dispatch packets
// (true: the lookups ran over target windows, k_sigma_tw)
bool launch_tcurve(hipStream_t s, TransitDev& tr, RunSlot& rs, int32_t nsig, bool msp, hipEvent_t ev_sig0,
                   hipEvent_t ev_sig1, hipEvent_t ev_tb0, hipEvent_t ev_tb1);
void launch_tau_mol(hipStream_t s, TransitDev& tr, RunSlot& rs, int32_t na, dim3 g, int32_t ppg);
void launch_mol_gt(hipStream_t s, const MolSlotDev& md);
void launch_rm_fout(hipStream_t s, TransitDev& tr);
void launch_tau_rm(hipStream_t s, TransitDev& tr, RunSlot& rs, int32_t na, hipEvent_t* ev);
double reduce_max(hipStream_t s, const double* v, int64_t n, double* scratch_dev);
// prom_gridded_density (prom_fn.hip)
void launch_gridded(hipStream_t s, const double* g, int32_t nx, int32_t ny, int32_t nz, int64_t n,
                    const double* px, const double* py, const double* pz, double* out);
// k_sigma_tw (prom_tw.hip): the lookups + curves over the problem's target windows (tr.tw_ok)
void launch_sigma_tw(hipStream_t s, TransitDev& tr, int32_t nsig, int32_t deg, const TcArgs& ta, hipEvent_t ev0,
                     hipEvent_t ev1);
// ... per set after new windows: mark the exact guesses (SigSeg kind |= 4)
void launch_tw_exact(hipStream_t s, TransitDev& tr, int32_t nsig);
// target windows of the Doppler-shifted lookups (prom_window.hip): false when the inputs do not allow them
bool build_target_windows(const double* wav, int64_t n_wav, const double* shift, int32_t n_rows,
                          const std::vector<const std::vector<double>*>& tabs, int32_t lds, int32_t lamcap,
                          int32_t rowcap, int64_t pmax, std::vector<SigSeg>& seg_out, std::vector<int32_t>& row_out,
                          std::vector<int32_t>& lam_out, int32_t& n_win);
// AtomTable::rec from a table's x and y, and the per-interval |a| bounds (prom_fn.hip)
void launch_table_recs(hipStream_t s, const double* x, const double* y, int64_t n, double4* rec, double* amax);
void launch_scatter(hipStream_t s, const char* base, const ScatterDesc* d, int32_t n);
// per phase: sum / count of R over the band-selected wavelengths, max of R over all (prom_transit_band_stats)
void launch_band_stats(hipStream_t s, const double* R, const double* wav, int32_t n_orb, int64_t n_wav,
                       int32_t n_bands, const double* bounds, double* sum, int64_t* count, double* mx);
// Star.getFstarIntegrated with rotation: the disk-integrated stellar flux per wavelength (prom_fn.hip)
void launch_star_disk(hipStream_t s, const SigTabDev& tb, const double* shift, const double* clv, const double* rho,
                      int32_t n_cells, double dphi, double drho, const double* wav, int64_t n_wav, double* out);

}  // namespace prom
