/*
 * prom_hip.h -- C-ABI of libprom_hip.so, the MI355X (gfx950) transit radiative-transfer core.
 *
 * The reference (CrazeXD/Prometheus) is pure Python with a duck-typed plugin protocol and no
 * FFI.  Each entry point below replaces one function (or one fused group of functions) on its
 * per-(orbital phase, wavelength) optical-depth path; the file:line it replaces is cited next to
 * it (paths relative to the reference tree).  A Python binding over ctypes lives in
 * prometheus_amd/_native.py; the stub a maintainer would add to the reference is in INTEGRATION.md.
 *
 * Conventions
 *   - Plain C types only: int32_t/int64_t sizes, double arrays (IEEE binary64, C order).
 *   - Every function returns PROM_OK (0) or a negative prom_status; the message of the last failure
 *     on a context is prom_last_error(ctx).  No exception crosses the ABI.
 *   - Host pointers passed in are read during the call only (inputs are copied to device memory
 *     owned by the context); output pointers are host buffers the caller owns.
 *   - One context per device.  Calls on different contexts may run concurrently from different host
 *     threads; a context is not re-entrant.  The library keeps no global mutable state.
 */
#ifndef PROM_HIP_H
#define PROM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PROM_ABI_VERSION 6

typedef struct prom_ctx prom_ctx;

enum prom_status {
  PROM_OK = 0,
  PROM_E_ARG = -1,      /* invalid argument (shape, null pointer, unknown id/kind) */
  PROM_E_HIP = -2,      /* HIP runtime error (device missing, launch failure, ...) */
  PROM_E_NOMEM = -3,    /* device allocation failed */
  PROM_E_STATE = -4     /* call out of order (e.g. prom_transit_run before prom_transit_set) */
};

/* ---- context ------------------------------------------------------------------------------- */
int32_t prom_abi_version(void);
int32_t prom_device_count(int32_t* count);
int32_t prom_create(int32_t device, prom_ctx** out);
void prom_destroy(prom_ctx* ctx);
const char* prom_last_error(const prom_ctx* ctx);
int32_t prom_synchronize(prom_ctx* ctx);

/* ---- log-sigma lookup tables ----------------------------------------------------------------
 * A table is the (x, log10(sigma + offset)) pair that the reference stores in an interp1d object
 * (AtmosphericConstituent.constructLookupFunction, gasProperties.py:694-715).  Tables live in
 * device memory, identified by an id local to the context. */

/* Upload a precomputed table (x strictly as given, must be non-decreasing). */
int32_t prom_table_upload(prom_ctx* ctx, int64_t n, const double* x, const double* log_sigma,
                          double offset, int32_t* table_id);

/* Build the table on the device: sigma(x) = sum over lines, in the given order, of
 *   (pi e^2 / (m_e c)) f_l * voigt_profile(c/x - c/lambda_l, sigma_v/lambda_l, gamma_l)
 * then log10(sigma + offset).  Replaces calculateVoigtProfile + constructLookupFunction
 * (gasProperties.py:672-715); line_coef[l] = (pi e^2/(m_e c)) * f_l computed by the caller in
 * the reference's evaluation order.  log_sigma_out (host, n) may be NULL. */
int32_t prom_table_build_voigt(prom_ctx* ctx, int64_t n, const double* x, int32_t n_lines,
                               const double* line_wavelength, const double* line_gamma,
                               const double* line_coef, double sigma_v, double c_light,
                               double offset, int32_t* table_id, double* log_sigma_out);

/* sigma(x) itself (no log, no table): calculateVoigtProfile (gasProperties.py:672-692). */
int32_t prom_voigt_sigma(prom_ctx* ctx, int64_t n, const double* x, int32_t n_lines,
                         const double* line_wavelength, const double* line_gamma,
                         const double* line_coef, double sigma_v, double c_light,
                         double* sigma_out);

/* out[i] = 10^(interp(targets[i], table)) - offset with numpy.interp semantics (clamping, exact
 * node hits): n_interp_log (gasProperties.py:34-51) / AtmosphericConstituent.getSigmaAbs (:727-735). */
int32_t prom_table_lookup(prom_ctx* ctx, int32_t table_id, int64_t n_targets, const double* targets,
                          double* out);

/* Release a table's device memory; its id is reused by a later upload.  The reference drops its
 * interp1d objects with the constituent (gasProperties.py:694-715, :34-51 builds one per call); a
 * transit problem set on this context that reads the table is invalidated (prom_transit_run then
 * fails with PROM_E_STATE until prom_transit_set is called again). */
int32_t prom_table_free(prom_ctx* ctx, int32_t table_id);
/* Live tables on the context (atomic, molecular) and the device bytes they hold. */
int32_t prom_table_count(prom_ctx* ctx, int32_t* n_atomic, int32_t* n_molecular, int64_t* device_bytes);

/* ---- molecular tables (MolecularConstituent, gasProperties.py:765-818) ----------------------
 * Axes in the reference's units after its conversions: P [dyn cm^-2] (= p[Pa] * 10), T [K],
 * wavelength [cm] (= 1/bin_edges reversed, increasing); log_sigma[n_p][n_t][n_w] = log10(xsec + offset)
 * on those axes.  Lookup is trilinear in (P, T, wavelength) with RegularGridInterpolator(
 * bounds_error=False, fill_value=log10(offset)) semantics; P is clipped below at 1e-4. */
int32_t prom_molecular_upload(prom_ctx* ctx, int32_t n_p, const double* P, int32_t n_t, const double* T,
                              int64_t n_w, const double* wavelength, const double* log_sigma,
                              double offset, int32_t* table_id);
/* getSigmaAbs: sigma[c][x][w] for P[c][x], fixed T, wavelength[c][w] (gasProperties.py:789-818). */
int32_t prom_molecular_sigma(prom_ctx* ctx, int32_t table_id, int64_t n_chords, int32_t n_x,
                             const double* P, double T, int64_t n_wav, const double* wavelength,
                             double* sigma_out);
/* Release a molecular table (see prom_table_free). */
int32_t prom_molecular_free(prom_ctx* ctx, int32_t table_id);

/* ---- density scenarios (calculateNumberDensity, gasProperties.py:143-516) ------------------- */
enum prom_density_kind {
  PROM_DENSITY_BAROMETRIC = 1,  /* :143-161  p = {n_0, R, H}                                     */
  PROM_DENSITY_HYDROSTATIC = 2, /* :185-204  p = {n_0, R, G*mu*M, k_B*T, Jeans_0}                */
  PROM_DENSITY_POWERLAW = 3,    /* :228-244, :311-330, :356-374  p = {n_0, R, q} (planet or moon) */
  PROM_DENSITY_TORUS = 4,       /* :491-516  p = {n_0, a_torus, 4*H_torus, H_torus}              */
  PROM_DENSITY_TABULATED = 5,   /* any other plugin: n(c, x) evaluated by the caller              */
  PROM_DENSITY_GRIDDED = 6      /* SerpensExosphere :548-601: scipy RegularGridInterpolator (linear,
                                   bounds_error) of a 3-D grid at (x - body_x, y - body_y, z);
                                   p = {n_gx, n_gy, n_gz}, grid in prom_scenario.n_tabulated as
                                   [gx[n_gx], gy[n_gy], gz[n_gz], values[n_gx][n_gy][n_gz]]        */
};

typedef struct prom_density_model {
  int32_t kind;
  int32_t reserved;
  double p[8];   /* scalars precomputed on the host in the reference's evaluation order */
} prom_density_model;

/* n[c][x] at chords with sky-plane coordinates (y[c], z[c]) = rho*(sin phi, cos phi) and density
 * centre (body_x[c], body_y[c]) (the planet's or moon's getPosition at that chord's phase). */
int32_t prom_number_density(prom_ctx* ctx, const prom_density_model* model, int32_t n_x,
                            const double* x, int64_t n_chords, const double* y, const double* z,
                            const double* body_x, const double* body_y, double* n_out);

/* SerpensExosphere.InterpolatedDensity (gasProperties.py:583-601; scipy RegularGridInterpolator, method
 * linear): out[i] = trilinear value of values[n_gx][n_gy][n_gz] on the ascending axes gx, gy, gz at
 * (px[i], py[i], pz[i]), in scipy's corner order.  A point outside the grid in any dimension gives NaN
 * (the reference raises: bounds_error=True). */
int32_t prom_gridded_density(prom_ctx* ctx, int32_t n_gx, const double* gx, int32_t n_gy, const double* gy,
                             int32_t n_gz, const double* gz, const double* values, int64_t n_points,
                             const double* px, const double* py, const double* pz, double* out);

/* ---- the fused transit integrator (Transit.sumOverChords, gasProperties.py:1160-1258, with
 *      Atmosphere.getLOSopticalDepth_Batch :885-956 and the density / sigma lookups inside) ----- */
typedef struct prom_constituent {
  int32_t table_id;      /* atomic: lookup-table id; molecular: molecular-table id */
  int32_t is_molecule;
  double chi;            /* mixing ratio (1.0 for exospheres) */
} prom_constituent;

typedef struct prom_scenario {
  prom_density_model density;
  const double* body_x;        /* [n_orb] density centre per phase (planet or moon)          */
  const double* body_y;        /* [n_orb]                                                     */
  const double* shift;         /* [n_orb] Doppler factor per phase (constants.py:31-45)       */
  const double* n_tabulated;   /* TABULATED: n[c][x] in the reference's chord order
                                  (c = ip * n_orb + o, geometryHandler.py:202-207);
                                  GRIDDED: the packed axes and values (prom_density_kind)      */
  double T;                    /* molecular constituents: lookup temperature                  */
  int32_t n_constituents;
  int32_t reserved;
  const prom_constituent* constituents;
} prom_scenario;

typedef struct prom_transit_problem {
  int64_t n_wav;               /* wavelengths of this shard                                   */
  const double* wavelength;    /* [n_wav] cm                                                  */
  int32_t n_pr;                /* chord positions per phase = phi_steps * rho_steps           */
  int32_t n_orb;               /* orbital phases                                              */
  const double* chord_y;       /* [n_pr] rho sin(phi), phi-major order                        */
  const double* chord_z;       /* [n_pr] rho cos(phi)                                         */
  const double* chord_fout;    /* [n_pr] F_out = rho * F_star * clv (flat star)               */
  int32_t n_x;                 /* line-of-sight samples                                       */
  int32_t n_scenarios;
  const double* x;             /* [n_x] cm                                                    */
  double delta_x;
  const double* planet_y;      /* [n_orb] planet y per phase: blocked if sqrt(dy^2+z^2) < R   */
  double planet_R;
  int32_t n_moons;
  int32_t reserved;
  const double* moon_y;        /* [n_moons][n_orb]: blocked if dy^2 + z^2 < R_m^2             */
  const double* moon_R;        /* [n_moons]                                                   */
  const prom_scenario* scenarios;
  double cull_tau;             /* chords whose tau upper bound is below this are transparent
                                  (exp(-tau) == 1 to the last ulp); <= 0 selects 2^-60       */
  int32_t options;             /* PROM_OPT_* bit set                                          */
  int32_t reserved2;
  double k_B;                  /* Boltzmann constant for P = n k_B T of molecular lookups
                                  (<= 0: the reference's 1.381e-16, constants.py:17)          */
  /* Stellar spectrum (gasProperties.py:1180-1219): with has_star != 0 the flux of chord c at
   * wavelength w is F = rho_c * (F_star(lambda_w / s_c) * clv_c), F_star(t) = 10^interp(t, star
   * table) (n_interp_log with offset 0, :34-51) and s_c = calculateDopplerShift(vsini rho_c / R_star
   * cos(phi_c - phi_rot)) (the Rossiter-McLaughlin shift, :1183-1184); chord_fout is then unused.
   * has_star == 0 keeps the flat star (F_star = 1, :1210-1211).  Atomic constituents only. */
  int32_t has_star;
  int32_t star_table;          /* table id (prom_table_upload of Fstar_function.x, .y; offset 0) */
  const double* chord_rho;     /* [n_pr] rho                                                  */
  const double* chord_clv;     /* [n_pr] 1 - u1 (1 - mu) - u2 (1 - mu)^2                       */
  const double* chord_star_shift;  /* [n_pr] s_c                                              */
} prom_transit_problem;

/* prom_transit_problem.options */
#define PROM_OPT_OCML_EXP 1    /* use the ocml exp() in the tau kernel instead of the table-driven exp */
#define PROM_OPT_NO_MERGE 2    /* integrate every active chord (no merging of equal-column chords) */
#define PROM_OPT_NO_WINDOW 4   /* evaluate exp(-tau) for every record at every wavelength (no saturated-
                                  head skip, no tail moments; see DESIGN.md "windowed integration") */
#define PROM_OPT_DOPPLER_ROWS 8 /* one Doppler sigma row per orbital phase even when the phases' factors are
                                  equal (a phase shard of a Doppler-shifted problem: the full problem's path,
                                  so its R rows are the full run's bit for bit) */

typedef struct prom_transit_stats {
  double ms_total;             /* device time of the last prom_transit_run (hipEvents)        */
  double ms_density;           /* density + column-density + culling kernels                  */
  double ms_sigma;             /* sigma resample kernel                                       */
  double ms_tau;               /* fused tau -> exp -> disk-sum kernel                         */
  int64_t active_chords;       /* chord-phase pairs integrated (all phases)                   */
  int64_t transparent_chords;  /* chord-phase pairs folded in as exp(-tau) = 1                */
  int64_t blocked_chords;
  int64_t chord_lambda_evals;  /* active_chords * n_wav                                        */
  int64_t tau_records;         /* chord records the tau kernel integrates (after merging)     */
  int64_t exp_evals;           /* exp evaluations of the fused kernel (counted on the device:
                                  the windowed kernel evaluates only the records of each
                                  wavefront's tau window; tau_records * n_wav without windows;
                                  molecular problems add the 10^v of every in-table sample)   */
  int32_t tau_kernel_variant;  /* which integration path the run took: tens = path, units = effective atomic
                                  species the path's kernels see (1 when species are merged into one absorber,
                                  0 when more than 4).  Tens (prom_transit.hip launch_transit):
                                    0  exact chord-order validation kernel k_tau with the ocml exp
                                       (PROM_OPT_OCML_EXP, and phases with a non-finite column);
                                    1  k_tau with the table exp (generic path; with molecular constituents:
                                       k_mol_list + k_tau_mol);
                                    2  windowed integration k_tau_w (k_order windows, per-tile records);
                                    3  planned windowed integration k_tau_p (k_order + k_windows heavy lists);
                                    4  stellar spectrum / CLV / RM rotation k_tau_rm;
                                    8  transmission curves, the default for one effective absorber:
                                       k_columns8 -> k_tc_build -> k_sigma_tc (prom_tcurve.hip; no orbital
                                       Doppler shift between the phases, one phase, or coarse tables);
                                    9  transmission curves with the Doppler-shifted lookups over target
                                       windows: k_columns8 -> k_tc_build -> k_sigma_tw (prom_tw.hip)       */
  int32_t tau_kernel_variant_exact_phases;  /* phases integrated on the exact (ocml) path because a
                                               column density was not finite                      */
} prom_transit_stats;

/* Copy a problem to the device (all host arrays are read during the call). */
int32_t prom_transit_set(prom_ctx* ctx, const prom_transit_problem* problem);
/* Run the integrator on the device; R stays in device memory.  stats may be NULL (with stats the
 * call waits for the run).  Runs are asynchronous: consecutive runs of a problem on the atomic paths
 * rotate over PROM_PIPELINE (default 4) internal streams and work-buffer slots, so the kernels of one run
 * (on the default path k_columns8 -> k_tc_build -> k_sigma_tc) overlap those of the runs before it; each
 * run is complete and independent.  prom_transit_result, prom_synchronize and prom_transit_set wait for
 * all of them. */
int32_t prom_transit_run(prom_ctx* ctx, prom_transit_stats* stats);
/* Copy R[n_orb][n_wav] (row-major) of the last run to a host buffer.  A buffer from prom_host_alloc
 * takes one DMA at the link rate; any other buffer is filled through the context's pinned staging. */
int32_t prom_transit_result(prom_ctx* ctx, double* R_out);

/* Page-locked host memory for results (ABI 4).  Process-wide pool, independent of contexts: a freed
 * buffer is kept for the next request of a similar size (size <= capacity <= 2 size), so a caller that
 * takes a fresh output array per call pays neither hipHostMalloc nor page faults.  Pinned bytes (in use +
 * cached) are capped at PROM_PINNED_CAP_MB (default 4096): past the cap PROM_E_NOMEM, and the caller falls
 * back to ordinary memory.  Replaces the reference's np.zeros result arrays (gasProperties.py:1165-1166). */
int32_t prom_host_alloc(int64_t bytes, void** out);
/* Return a prom_host_alloc buffer to the pool (PROM_E_ARG for any other pointer). */
int32_t prom_host_free(void* p);
/* Column densities N[s][o][ip] of the last run (atomic constituents in scenario order); testing aid. */
int32_t prom_transit_columns(prom_ctx* ctx, double* N_out);

/* Band statistics of the last run's R on the device, for light curves (the band-averaged transit
 * depth of mainRetrieval.py:76-93) without copying R to the host.  Phase o selects the wavelengths
 * with bounds[o][b][0] <= lambda <= bounds[o][b][1] for any band b; sum_out[o] is the sum of R over
 * them, count_out[o] their number and max_out[o] the maximum of R over ALL wavelengths of the problem
 * (NaN if any R is NaN, like numpy.max).  Over wavelength shards the sums and counts add and the
 * maxima combine with max; the light curve is (sum / count) / max. */
int32_t prom_transit_band_stats(prom_ctx* ctx, int32_t n_bands, const double* bounds, double* sum_out,
                                int64_t* count_out, double* max_out);

/* Per-kernel device durations of the transit path (ABI 5; ids 5 and 6 since ABI 6): n_runs runs of the current problem, one at a
 * time (one slot, no second stream; the stream waits after every run), each kernel timed by start/stop
 * events on its own dispatch packet (groups of kernels: the first start to the last stop).  ms_out[k] is
 * the mean duration in milliseconds of kernel k (prom_kernel_id), NaN when the path does not launch it.
 * What rocprofv3 --kernel-trace reports for one slot in flight; measurement aid for bench.py. */
enum prom_kernel_id {
  PROM_K_COLUMNS = 0,   /* densities, column densities and culling: k_columns8 (atomic paths); k_ntot +
                           k_mol_prep + k_columns (molecular and generic paths)                        */
  PROM_K_SIGMA = 1,     /* Doppler cross-section rows of the windowed paths: k_sigma_poly / k_sigma_rows */
  PROM_K_ORDER = 2,     /* per-phase chord ordering: k_order (windowed paths), k_chords (generic and
                           molecular paths)                                                            */
  PROM_K_WINDOWS = 3,   /* tile windows and heavy-entry lists: k_windows (planned windowed path)        */
  PROM_K_TAU = 4,       /* the integration kernel: k_tau / k_tau_w / k_tau_p / k_tau_rm / k_mol_list +
                           k_tau_mol                                                                   */
  PROM_K_TC_BUILD = 5,  /* transmission-curve path: every phase's curve T_o, k_tc_build                 */
  PROM_K_SIGMA_TC = 6,  /* transmission-curve path: sigma at each phase's Doppler shift and R = T_o(Y),
                           k_sigma_tc                                                                  */
  PROM_K_COUNT = 7      /* length of prom_transit_kernel_ms's ms_out                                   */
};
int32_t prom_transit_kernel_ms(prom_ctx* ctx, int32_t n_runs, double* ms_out);

/* Disk-integrated stellar flux of a rotating star (ABI 5).  Replaces the rotating branch of
 * Star.getFstarIntegrated (celestialBodies.py:299-311, through calculateRM :226-240 and calculateCLV
 * :212-224): for every wavelength, the n_cells disk cells in the reference's loop order (phi outer, rho
 * inner) are accumulated one after the other,
 *   out[w] += (((10^interp(wavelength[w] / shift[c]) * clv[c]) * dphi) * drho) * rho[c],
 * interp = numpy.interp over the star table (offset 0).  The caller gives each cell's Doppler factor
 * (calculateDopplerShift of the surface velocity) and CLV factor.  A target outside the table is an
 * error (PROM_E_ARG), as the reference's interp1d(bounds_error=True) raises. */
int32_t prom_star_disk_flux(prom_ctx* ctx, int32_t star_table, int32_t n_cells, const double* shift,
                            const double* clv, const double* rho, double dphi, double drho, int64_t n_wav,
                            const double* wavelength, double* out);

/* Live per-run timing of the tau kernel without per-run synchronisation: between prom_timing_begin
 * and prom_timing_end every timed prom_transit_run carries a HIP event pair (the ordering kernel's
 * completion -> the tau kernel's completion) and, for the planned tau kernel k_tau_p, device-clock
 * stamps of its workgroups; prom_timing_end waits for them and returns ms[run][4] =
 * {NaN, NaN, tau_events, tau_device} for up to max_runs runs (n_runs receives the count).
 * tau_events includes the tau kernel's dispatch behind the ordering kernel; tau_device is the span
 * from its first workgroup's start to its last workgroup's end (NaN for other tau kernels).  Stage times of a single run come from prom_transit_run's stats.
 * prom_timing_stride(ctx, k) (k >= 1, default 1, kept until changed) times only every k-th run of the
 * window: events on a dispatch cost the host ~13 us, more than a run's GPU time, so a throughput
 * measurement samples the kernel durations instead of timing every run. */
int32_t prom_timing_begin(prom_ctx* ctx);
int32_t prom_timing_end(prom_ctx* ctx, int32_t max_runs, double* ms, int32_t* n_runs);
int32_t prom_timing_stride(prom_ctx* ctx, int32_t stride);

#ifdef __cplusplus
}
#endif

#endif /* PROM_HIP_H */
