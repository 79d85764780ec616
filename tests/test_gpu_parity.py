"""GPU parity: the HIP path (through the C-ABI of libprom_hip.so) against the golden vectors
of the reference and against the CPU oracle.  Marked ``gpu``: runs on an MI355X only.

Tolerances (float64 throughout):
  * R(phase, wavelength): 1e-10 relative (the north-star bar); observed ~1e-14.
  * sigma tables (log10 sigma): 1e-12 absolute in log space -- the Voigt function is our own
    Faddeeva implementation (faddeeva.h, <= 2e-15 vs mpmath) against scipy's (~2e-14).
  * densities, lookups: 1e-13 relative (libm vs ocml exp/pow/sin differ by an ulp).
"""
import json
import os

import numpy as np
import pytest

from oracle import prom_oracle as O

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
R_TOL = 1e-10


def load(name):
    return np.load(os.path.join(G, name + ".npz"))


@pytest.fixture(scope="module")
def dev():
    from prometheus_amd import _native
    return _native.get_device(0)


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    r[(a == b)] = 0.0
    return float(np.max(r)) if r.size else 0.0


def test_native_loaded(dev):
    from prometheus_amd import _native
    assert _native.device_count() >= 1
    assert dev.h


def test_table_lookup_kats(dev):
    d = load("interp_kats")
    tid = dev.table_upload(d["xg"], d["yg"], 1e-50)
    out = dev.table_lookup(tid, d["t"])
    assert rel(out, d["out"]) < 1e-14
    # the interpolated log value itself is bitwise numpy.interp
    tid0 = dev.table_upload(d["xg"], d["yg"], 0.0)
    v = np.log10(dev.table_lookup(tid0, d["t"]))
    assert np.max(np.abs(v - np.interp(d["t"], d["xg"], d["yg"]))) < 1e-13


def test_voigt_tables(dev):
    from prometheus_amd import constants as const
    from prometheus_amd import gasProperties as gp
    d = load("cross_sections")
    i = 0
    while "case%d_x" % i in d:
        meta = json.loads(str(d["case%d_meta" % i]))
        sp = const.AvailableSpecies().findSpecies(meta["species"])
        con = gp.AtmosphericConstituent(sp, 1., meta["sigma_v"])
        wg = gp.WavelengthGrid(meta["lower_w"], meta["upper_w"], 2e-8, 5e-9, 2e-10)
        lf = con.constructLookupFunction(wg)
        assert np.array_equal(lf.x, d["case%d_x" % i])
        assert np.max(np.abs(lf.y - d["case%d_y" % i])) < 1e-12, i
        sig = con.calculateVoigtProfile(d["case%d_sigma_direct_w" % i])
        ref = d["case%d_sigma_direct" % i]
        assert rel(sig, ref) < 1e-12 or (np.all(ref == 0) and np.all(sig == 0)), i
        i += 1


def test_density_plugins(dev):
    from prometheus_amd import celestialBodies as cb
    from prometheus_amd import constants as const
    from prometheus_amd import gasProperties as gp
    d = load("density")
    planet = cb.AvailablePlanets().findPlanet("WASP-49b")
    m0, mR, ma = d["moon_params"]
    moon = cb.Moon(m0, mR, ma, planet)
    models = {
        "barometric": gp.BarometricAtmosphere(3000., 1e4, 2.3 * const.amu, planet),
        "hydrostatic": gp.HydrostaticAtmosphere(1500., 1e5, 2.3 * const.amu, planet),
        "powerLawAtm": gp.PowerLawAtmosphere(3000., 1e-3, 6., planet),
        "powerLawExo": gp.PowerLawExosphere(1e33, 4.5, planet),
        "exomoon": gp.MoonExosphere(1e32, 3.34, moon),
        "torus": gp.TorusExosphere(1e33, 2 * planet.R, 5e5, planet),
    }
    for k, m in models.items():
        n = m.calculateNumberDensity(d["x"], d["phi"], d["rho"], d["orb"])
        assert n.shape == d[k].shape
        assert rel(n, d[k]) < 1e-12, (k, rel(n, d[k]))


def test_molecular_kat(dev):
    d = load("molecular_kat")
    P = d["tab_p"] * 10.
    W = 1. / d["tab_bin_edges"][::-1]
    V = np.log10(d["tab_xsecarr"][:, :, ::-1] + 1e-50)
    tid = dev.molecular_upload(P, d["tab_t"], np.ascontiguousarray(W), np.ascontiguousarray(V), 1e-50)
    sig = dev.molecular_sigma(tid, d["P"], float(d["T"]), d["wav"])
    assert rel(sig, d["sigma"]) < 1e-12


def _product_transit(cfg):
    from prometheus_amd import gasProperties as gp
    from prometheus_amd import setupfile
    gp.register_molecular_table("H2O", O.synthetic_molecular_table(n_nu=2001))
    return setupfile.build_transit(cfg)


@pytest.mark.parametrize("name", ["C1", "C2r", "C3r", "C4r", "C5r", "exomoon"])
def test_transit_golden(dev, name):
    d = load("transit_" + name)
    cfg = json.loads(str(d["config"]))
    tr = _product_transit(cfg)
    assert np.array_equal(tr.wavelength, d["wavelength"])
    R = tr.sumOverChords(devices=[0])
    err = rel(R, d["R"])
    print("%s: max rel err %.3e over %d points, stats %s" % (name, err, R.size, tr.last_stats[-1]))
    assert err < R_TOL


@pytest.mark.parametrize("name", ["C2r", "C3r", "C4r", "C5r"])
def test_transit_ocml_exp_mode(dev, name):
    """The validation build of the tau kernel (ocml exp) agrees with the table exp and the reference; on the
    molecular path (C5r) the ocml build is checked against the reference's golden R at 1e-12, an independent check
    of the per-set T-folded table k_mol_gt that both exp modes read."""
    from prometheus_amd import _native
    d = load("transit_" + name)
    tr = _product_transit(json.loads(str(d["config"])))
    R_tab = tr.sumOverChords(devices=[0])
    R_ocml = tr.sumOverChords(devices=[0], options=_native.OPT_OCML_EXP)
    assert rel(R_ocml, d["R"]) < R_TOL and rel(R_tab, d["R"]) < R_TOL
    assert rel(R_tab, R_ocml) < 1e-13
    if name == "C5r":
        assert rel(R_ocml, d["R"]) < 1e-12


def test_molecular_mirror_merging(dev, monkeypatch):
    """Mirror-image chords (z -> -z) with equal molecular sample lists are integrated once with the summed weight
    (k_mol_list): R with merging agrees with the unmerged R to 1e-13 and with the reference's golden R."""
    d = load("transit_C5r")
    tr = _product_transit(json.loads(str(d["config"])))
    tr.collect_stats = True
    R_m = tr.sumOverChords(devices=[0])
    ev_m = tr.last_stats[-1]["exp_evals"]
    monkeypatch.setenv("PROM_MOL_MIRROR", "0")
    R_u = tr.sumOverChords(devices=[0])
    ev_u = tr.last_stats[-1]["exp_evals"]
    print("C5r mirror merging: rel diff %.3e, vs golden %.3e / %.3e, evaluations %d -> %d"
          % (rel(R_m, R_u), rel(R_m, d["R"]), rel(R_u, d["R"]), ev_u, ev_m))
    assert ev_m < ev_u   # (pairs were merged: fewer 10^v evaluations)
    assert rel(R_m, R_u) < 1e-13
    assert rel(R_m, d["R"]) < R_TOL and rel(R_u, d["R"]) < R_TOL


def test_molecular_lds_stage_matches_global_reads(dev, monkeypatch):
    """k_tau_mol's LDS stage of the G records returns the global records' values: R bitwise with the stage
    disabled (PROM_MOL_STAGE=0, every sample read from global memory)."""
    d = load("transit_C5r")
    tr = _product_transit(json.loads(str(d["config"])))
    R_s = tr.sumOverChords(devices=[0])
    monkeypatch.setenv("PROM_MOL_STAGE", "0")
    R_g = tr.sumOverChords(devices=[0])
    assert np.array_equal(R_s, R_g)
    assert rel(R_s, d["R"]) < R_TOL


def test_molecular_pipelined_runs(dev):
    """Molecular runs rotate over the pipeline slots (per-slot samples and lists): every run's R is the same, with
    the runs issued back to back (several in flight on the slots' streams) before one result is read."""
    d = load("transit_C5r")
    tr = _product_transit(json.loads(str(d["config"])))
    R = [tr.sumOverChords(devices=[0]) for _ in range(3)]
    for r in R[1:]:
        assert np.array_equal(r, R[0])
    assert rel(R[0], d["R"]) < R_TOL
    host = tr._host_inputs()
    prob = tr._problem(dev, host, 0, len(tr.wavelength), 0.0)
    dev.transit_set(prob)
    for _ in range(7):   # (> the 4 pipeline slots: every slot reused while earlier runs may still be in flight)
        dev.transit_run()
    Rp = dev.transit_result()
    assert np.array_equal(Rp, R[0])


@pytest.mark.parametrize("name", ["C1", "C2r", "C4r", "exomoon"])
def test_chord_merging(dev, name, monkeypatch):
    """Merging chords with equal (2^-40) column densities moves R by <= 2^-40/e.  Checked with
    every active chord sorted (PROM_NO_TAIL_SPLIT): always-tail chords are otherwise left unsorted behind
    the others, where equal neighbours are not adjacent (test_tail_split)."""
    monkeypatch.setenv("PROM_TCURVE", "0")   # the windowed path (k_order); transmission curves: test_gpu_tcurve.py
    from prometheus_amd import _native
    monkeypatch.setenv("PROM_NO_TAIL_SPLIT", "1")
    d = load("transit_" + name)
    tr = _product_transit(json.loads(str(d["config"])))
    R_m = tr.sumOverChords(devices=[0])
    st_m = tr.last_stats[-1]
    R_n = tr.sumOverChords(devices=[0], options=_native.OPT_NO_MERGE)
    st_n = tr.last_stats[-1]
    # merging moves R by <= 2^-40/e; both runs are windowed (<= 2^-40/24 + e^-40 each vs full evaluation)
    assert np.max(np.abs(R_m - R_n)) <= 2.0 ** -40 / np.e + 2 * (2.0 ** -40 / 24 + np.exp(-40.0)) + 1e-15
    assert st_n["tau_records"] == st_n["active_chords"]
    assert st_m["tau_records"] <= st_m["active_chords"]
    print(name, "records merged %d -> %d" % (st_m["active_chords"], st_m["tau_records"]))
    if name == "C1":   # one phase with the planet at the disk centre: whole rings merge
        assert st_m["tau_records"] * 10 < st_m["active_chords"]


@pytest.mark.parametrize("name", ["C1", "C2r", "C3r", "C4r", "exomoon"])
def test_tail_split(dev, name, monkeypatch):
    """k_order leaves chords with b Q_bound < the tail epsilon unsorted behind the sorted ones (their
    envelope is the threshold itself): R moves by no more than the windowed bound, and stays within the
    north-star tolerance of the reference."""
    monkeypatch.setenv("PROM_TCURVE", "0")   # the windowed path (k_order); transmission curves: test_gpu_tcurve.py
    d = load("transit_" + name)
    cfg = json.loads(str(d["config"]))
    R_s = _product_transit(cfg).sumOverChords(devices=[0])
    monkeypatch.setenv("PROM_NO_TAIL_SPLIT", "1")
    R_n = _product_transit(cfg).sumOverChords(devices=[0])
    assert np.max(np.abs(R_s - R_n)) <= 1e-13   # each run within 4e-14 of the full evaluation
    assert rel(R_s, d["R"]) < R_TOL


def test_sharding_bitwise(dev):
    """Wavelength shards (1, 2, 3 ways; emulated on one GPU) give bitwise-identical R."""
    d = load("transit_C2r")
    tr = _product_transit(json.loads(str(d["config"])))
    R1 = tr.sumOverChords(devices=[0])
    R2 = tr.sumOverChords(devices=[0, 0])
    R3 = tr.sumOverChords(devices=[0, 0, 0])
    assert np.array_equal(R1, R2) and np.array_equal(R1, R3)


def test_transit_c2_full_grid_sampled(dev):
    """Full C2 (190,205 wavelengths x 8 phases x 2,400 chords) on the GPU, checked against the
    oracle on a seeded sample of 600 wavelengths (R at one wavelength does not depend on the others)."""
    from prometheus_amd import configs
    cfg = configs.get("C2")
    tr = _product_transit(cfg)
    R = tr.sumOverChords(devices=[0])
    assert R.shape == (8, 190205)
    rng = np.random.default_rng(5)
    idx = np.sort(rng.choice(R.shape[1], 600, replace=False))
    scen, dop, grids = O.from_setup(cfg)
    tabs = O.build_tables(scen, grids)
    Ro = O.transit_depth(scen, dop, grids, tr.wavelength[idx], tabs)
    err = rel(R[:, idx], Ro)
    print("C2 sampled max rel err %.3e" % err)
    assert err < R_TOL
    assert np.all(np.isfinite(R)) and np.all((R > 0) & (R <= 1.0 + 1e-12))


@pytest.mark.parametrize("name", ["C1", "C2r", "C3r", "C4r", "exomoon"])
def test_windowed_integration(dev, name, monkeypatch):
    """Windowed integration (saturated-head skip + cubic tail moments) against full
    evaluation of every record: |dR| <= 2^-40/24 + e^-40 (+ rounding), and fewer exp evaluations."""
    monkeypatch.setenv("PROM_TCURVE", "0")   # the windowed path (k_order); transmission curves: test_gpu_tcurve.py
    from prometheus_amd import _native
    d = load("transit_" + name)
    tr = _product_transit(json.loads(str(d["config"])))
    R_w = tr.sumOverChords(devices=[0])
    st_w = tr.last_stats[-1]
    R_f = tr.sumOverChords(devices=[0], options=_native.OPT_NO_WINDOW)
    st_f = tr.last_stats[-1]
    bound = 2.0 ** -40 / 24 + np.exp(-40.0) + 1e-15
    diff = float(np.max(np.abs(R_w - R_f)))
    print(name, "window |dR| %.3e, exp evals %d -> %d" % (diff, st_f["exp_evals"], st_w["exp_evals"]))
    assert diff <= bound
    assert st_w["exp_evals"] <= st_f["exp_evals"]
    assert st_f["exp_evals"] == st_f["tau_records"] * R_f.shape[1]
    assert rel(R_w, d["R"]) < R_TOL


def test_windowed_no_merge_no_window_matches_reference(dev):
    """All four combinations of merging and windows agree with the reference on C2r."""
    from prometheus_amd import _native
    d = load("transit_C2r")
    tr = _product_transit(json.loads(str(d["config"])))
    for opt in (0, _native.OPT_NO_MERGE, _native.OPT_NO_WINDOW, _native.OPT_NO_MERGE | _native.OPT_NO_WINDOW):
        R = tr.sumOverChords(devices=[0], options=opt)
        assert rel(R, d["R"]) < R_TOL, opt


def _with_star(tr, star, x, F):
    hs = tr.planet.hostStar
    hs.addCLVparameters(star["u1"], star["u2"])
    hs.addRMparameters(star["vsini"], star["phi_rot"])
    hs.addFstarSpectrum(x, F)
    return tr


@pytest.mark.parametrize("name", ["rm_C1", "rm_C2r", "rm_exomoon"])
def test_stellar_spectrum_golden(dev, name):
    """Stellar spectrum with CLV and Rossiter-McLaughlin rotation (gasProperties.py:1180-1219) against
    the reference's own R; table exp and ocml exp; shards bitwise identical."""
    from prometheus_amd import _native, configs
    d = load(name)
    cfg = json.loads(str(d["config"]))
    star = json.loads(str(d["star"]))
    g = cfg["Grids"]
    x, F = configs.synthetic_star_spectrum(g["lower_w"], g["upper_w"])
    tr = _with_star(_product_transit(cfg), star, x, F)
    R = tr.sumOverChords(devices=[0])
    st = tr.last_stats[-1]
    err = rel(R, d["R"])
    print("%s: max rel err %.3e, stats %s" % (name, err, st))
    assert err < R_TOL
    assert st["tau_kernel_variant"] >= 40
    assert st["active_chords"] + st["transparent_chords"] + st["blocked_chords"] == R.shape[0] * tr.spatialGrid.phi_steps * tr.spatialGrid.rho_steps
    R_o = tr.sumOverChords(devices=[0], options=_native.OPT_OCML_EXP)
    assert rel(R_o, d["R"]) < R_TOL and rel(R, R_o) < 1e-13
    assert np.array_equal(R, tr.sumOverChords(devices=[0, 0, 0]))


def test_stellar_spectrum_fine_table_global_lookup(dev):
    """A stellar table too fine for the LDS slice (> 1024 nodes per workgroup) takes the global
    directory lookup; checked against the oracle."""
    from prometheus_amd import configs
    cfg = configs.get("C1")
    star = {"u1": 0.5, "u2": 0.1, "vsini": 8e6, "phi_rot": 2.0}
    g = cfg["Grids"]
    x, F = configs.synthetic_star_spectrum(g["lower_w"], g["upper_w"], step=5e-12)
    tr = _with_star(_product_transit(cfg), star, x, F)
    R = tr.sumOverChords(devices=[0])
    wav, orb, Ro = O.run_setup(cfg, None, star=dict(star, fstar=(x, np.log10(F))))
    assert np.array_equal(wav, tr.wavelength)
    assert rel(R, Ro) < R_TOL


def test_stellar_spectrum_clustered_nodes(dev):
    """A non-uniform stellar table (a coarse grid plus tight node clusters and repeated nodes) makes
    the slice directory's buckets crowded (bisection fallback); checked against the oracle."""
    from prometheus_amd import configs
    cfg = configs.reduced(configs.get("C2"), orbphase_steps=3, lower_w=5886e-8, upper_w=5894e-8,
                          res_low=5e-9, res_high=1e-10)
    star = {"u1": 0.3, "u2": 0.2, "vsini": 4e6, "phi_rot": 0.7}
    g = cfg["Grids"]
    x0, F0 = configs.synthetic_star_spectrum(g["lower_w"], g["upper_w"], step=5e-10)
    rng = np.random.default_rng(3)
    extra = np.concatenate([c + np.linspace(0, 2e-11, 100) for c in rng.uniform(x0[5], x0[-5], 4)])
    x = np.sort(np.concatenate([x0, extra, x0[100:103]]))          # three repeated nodes
    F = np.interp(x, x0, F0) * (1. + 0.2 * np.sin(x * 3e9))
    tr = _with_star(_product_transit(cfg), star, x, F)
    R = tr.sumOverChords(devices=[0])
    wav, orb, Ro = O.run_setup(cfg, None, star=dict(star, fstar=(x, np.log10(F))))
    assert np.array_equal(wav, tr.wavelength)
    assert rel(R, Ro) < R_TOL


@pytest.mark.parametrize("name", ["exomoon", "C2r"])
def test_band_lightcurve(dev, name):
    """Transit.bandLightcurve (device band reduction over R in HBM, mainRetrieval.py:76-93) against the
    oracle's light curve of the reference's R; sharded and with the spectrum returned."""
    d = load("transit_" + name)
    cfg = json.loads(str(d["config"]))
    tr = _product_transit(cfg)
    scen, _, _ = O.from_setup(cfg)
    ref = O.lightcurve(d["R"], d["wavelength"], d["orbphase"], scen[0].planet)
    lc1 = tr.bandLightcurve(devices=[0])
    lc2, R = tr.bandLightcurve(devices=[0, 0], return_spectrum=True)
    assert rel(lc1, ref) < R_TOL and rel(lc2, ref) < R_TOL
    assert rel(R, d["R"]) < R_TOL
    print(name, "light curve", lc1)


def test_many_los_samples_generic_columns(dev):
    """n_x > 64 takes the generic density / column kernels (k_ntot + k_columns) in front of the
    windowed tau kernel; checked against the oracle."""
    from prometheus_amd import configs
    cfg = configs.reduced(configs.get("C2"), orbphase_steps=3, lower_w=5886e-8, upper_w=5900e-8,
                          res_low=5e-9, res_high=1e-10)
    cfg["Grids"]["x_steps"] = 80
    tr = _product_transit(cfg)
    R = tr.sumOverChords(devices=[0])
    scen, dop, grids = O.from_setup(cfg)
    Ro = O.transit_depth(scen, dop, grids, tr.wavelength, O.build_tables(scen, grids))
    assert rel(R, Ro) < R_TOL


@pytest.mark.parametrize("name", ["C1", "C2r", "C3r", "C4r", "exomoon", "C2", "C3"])
def test_planned_tau_within_window_bound(dev, name, monkeypatch):
    """The planned tau kernel (k_tau_p: static (tile, 4-phase) wavefronts for light windows, heavy entries
    per 64-wavelength half with their own windows, long ones split into 64-record chunks over a workgroup)
    against k_tau_w (PROM_TAU_PLAN=0: one window per 128-wavelength tile, records summed in order).  Light
    tiles are bitwise equal (most points); heavy halves differ by at most the two windows' truncation bounds
    plus the chunked summation's rounding, and never evaluate more exponentials."""
    monkeypatch.setenv("PROM_TCURVE", "0")   # the windowed path (k_order); transmission curves: test_gpu_tcurve.py
    from prometheus_amd import configs
    if name in ("C2", "C3"):
        cfg = configs.get(name)
    else:
        cfg = json.loads(str(load("transit_" + name)["config"]))
    tr = _product_transit(cfg)
    monkeypatch.setenv("PROM_TAU_PLAN", "1")
    R_p = tr.sumOverChords(devices=[0])
    st_p = tr.last_stats[-1]
    monkeypatch.setenv("PROM_TAU_PLAN", "0")
    R_w = tr.sumOverChords(devices=[0])
    st_w = tr.last_stats[-1]
    print(name, "variants", st_p["tau_kernel_variant"], st_w["tau_kernel_variant"], "exp evals", st_p["exp_evals"])
    assert st_p["tau_kernel_variant"] // 10 == 3 and st_w["tau_kernel_variant"] // 10 == 2
    bound = 2 * (2.0 ** -40 / 24 + np.exp(-40.0)) + 1e-14
    assert np.max(np.abs(R_p - R_w)) <= bound
    assert st_p["exp_evals"] <= st_w["exp_evals"]
    # light tiles (windows of <= kHeavy records, nearly every tile) take the same records in the same order
    # on both kernels and are bitwise equal; only heavy halves (line cores) may differ
    diff = R_p != R_w
    assert np.count_nonzero(diff) <= diff.size // 2


@pytest.mark.parametrize("name", ["C2r", "C2"])
def test_species_merge(dev, name, monkeypatch):
    """Constituents of one density scenario collapse into one effective absorber (tau = N Y with
    Y = sum_s chi_s sigma_s): R agrees with the per-species integration to rounding (1e-13 relative)
    and with the reference to R_TOL; the merged run has one effective species: the transmission-curve path
    (variant 81) by default, the windowed path's variant 31 with PROM_TCURVE=0."""
    from prometheus_amd import configs
    cfg = configs.get("C2") if name == "C2" else json.loads(str(load("transit_" + name)["config"]))
    tr = _product_transit(cfg)
    monkeypatch.setenv("PROM_SPECIES_MERGE", "1")
    R_m = tr.sumOverChords(devices=[0])
    st_m = tr.last_stats[-1]
    monkeypatch.setenv("PROM_SPECIES_MERGE", "0")
    R_s = tr.sumOverChords(devices=[0])
    st_s = tr.last_stats[-1]
    print(name, "variants", st_m["tau_kernel_variant"], st_s["tau_kernel_variant"],
          "exp evals %d -> %d" % (st_s["exp_evals"], st_m["exp_evals"]), "max rel diff %.3e" % rel(R_m, R_s))
    assert st_m["tau_kernel_variant"] in (81, 91) and st_s["tau_kernel_variant"] == 32
    assert rel(R_m, R_s) < 1e-13
    if name != "C2":
        assert rel(R_m, load("transit_" + name)["R"]) < R_TOL
    monkeypatch.setenv("PROM_SPECIES_MERGE", "1")
    monkeypatch.setenv("PROM_TCURVE", "0")
    R_w = tr.sumOverChords(devices=[0])
    assert tr.last_stats[-1]["tau_kernel_variant"] == 31
    assert rel(R_w, R_s) < 1e-13


@pytest.mark.parametrize("plan", ["1", "0", "doppler", "tcurve", "tcurve_doppler"])
def test_nonfinite_columns_exact_path(dev, plan, monkeypatch):
    """A user density plugin (host-tabulated n(c, x)) with one infinite sample: that chord's column is
    inf, its phase takes the exact chord-order path (ocml exp, no windows), e^{-inf sigma} = 0 and
    inf * 0 = NaN where sigma == 0, as in the reference dataflow (oracle on the same tabulated input).
    Both the planned (k_tau_p) and the k_tau_w fast path."""
    import copy
    from prometheus_amd import configs
    # "doppler": orbital Doppler shift on, so the merged Na + K absorber takes the fused path (the tau kernel
    # looks sigma and the zero flags up itself)
    # fused rows (k_sigma_poly integrates the exact phase itself); "doppler_rows": the sigma-row path
    # "tcurve", "tcurve_doppler": the transmission-curve path (k_sigma_tc integrates the exact phase itself)
    tcurve = plan.startswith("tcurve")
    monkeypatch.setenv("PROM_TCURVE", "1" if tcurve else "0")
    monkeypatch.setenv("PROM_TAU_PLAN", "1" if (plan.startswith("doppler") or tcurve) else plan)
    cfg = configs.reduced(configs.get("C2"), orbphase_steps=3, lower_w=5886e-8, upper_w=5900e-8,
                          res_low=5e-9, res_high=1e-10)
    cfg["Fundamentals"]["DopplerOrbitalMotion"] = plan.startswith("doppler") or plan == "tcurve_doppler"
    tr = _product_transit(cfg)
    scen, dop, grids = O.from_setup(cfg)
    base = scen[0]
    cg = O.chord_grid(grids)
    x = O.x_axis(grids)
    col = O.number_density(base, x, cg[:, 0], cg[:, 1], cg[:, 2]).sum(axis=1)
    orbs = O.orbphase_axis(grids)
    pl = base.planet
    y, z = cg[:, 1] * np.sin(cg[:, 0]), cg[:, 1] * np.cos(cg[:, 0])
    blocked = np.sqrt((y - pl.a * np.sin(cg[:, 2])) ** 2 + z ** 2) < pl.R
    cand = np.where((cg[:, 2] == orbs[1]) & ~blocked)[0]
    k0 = cand[np.argmax(col[cand])]   # the unblocked chord of phase 1 with the largest column
    tphi, trho, torb = cg[k0]

    def fn(x_, phi_, rho_, orb_):
        n = np.array(O.number_density(base, x_, phi_, rho_, orb_), dtype=np.float64)
        m = (np.isclose(phi_, tphi, rtol=1e-12, atol=0) & np.isclose(rho_, trho, rtol=1e-12, atol=0) &
             np.isclose(orb_, torb, rtol=1e-12, atol=1e-15))
        n[m, 3] = np.inf
        return n

    tab = O.Scenario("tabulated", base.planet, {}, constituents=base.constituents, T=base.T, tabulated_fn=fn)
    Ro = O.transit_depth([tab], dop, grids, tr.wavelength, O.build_tables([tab], grids))
    d0 = tr.atmosphere.densityDistributionList[0]

    class Plug(type(d0)):
        def densityModel(self):
            raise NotImplementedError

        def calculateNumberDensity(self, x_, phi_, rho_, orb_):
            return fn(x_, phi_, rho_, orb_)

    p = copy.copy(d0)
    p.__class__ = Plug
    tr.atmosphere.densityDistributionList[0] = p
    R = tr.sumOverChords(devices=[0])
    st = tr.last_stats[-1]
    print("plan", plan, "exact phases", st["exact_phases"], "NaN points", int(np.isnan(Ro).sum()), "variant",
          st["tau_kernel_variant"])
    assert st["exact_phases"] == 1
    assert (st["tau_kernel_variant"] in (81, 91)) == tcurve
    assert np.array_equal(np.isnan(R), np.isnan(Ro))
    m = ~np.isnan(Ro)
    assert rel(R[m], Ro[m]) < R_TOL


def test_graph_replay_matches(dev, monkeypatch):
    """PROM_GRAPH=1: untimed fast-path runs replay one captured hipGraph per pipeline slot; every
    replayed run's R is bitwise the directly launched run's."""
    monkeypatch.setenv("PROM_GRAPH", "1")
    d = load("transit_C2r")
    tr = _product_transit(json.loads(str(d["config"])))
    host = tr._host_inputs()
    dev.transit_set(tr._problem(dev, host, 0, len(tr.wavelength), 0.0))
    dev.transit_run(stats=True)
    R0 = dev.transit_result()
    for _ in range(9):
        dev.transit_run()
        dev.synchronize()
        assert np.array_equal(dev.transit_result(), R0)
    assert rel(R0, d["R"]) < R_TOL


@pytest.mark.parametrize("name,merge", [("C3r", "1"), ("C3r", "0"), ("C4r", "1"), ("exomoon", "1"), ("C3", "1"),
                                        ("C3", "0"), ("C4", "1")])
def test_sigma_rows_bitwise(dev, name, merge, monkeypatch):
    """Orbital Doppler shift: the per-phase cross-section rows against the per-target directory lookups
    (PROM_SIGMA_ROWS=0: sigma_of, numpy.interp + exp10 per target).  The exp10 rows (k_sigma_rows, table
    slices staged in LDS per wavelength block; PROM_SIG_POLY=0) are bit-for-bit those lookups, merged
    (Y = sum_s chi_s sigma_s) and per species: R is identical.  The polynomial rows (k_sigma_poly, the
    default: E_k e^a with a degree-D Taylor polynomial over the tables' {x, 10^y, ln10 slope} records) move
    sigma by ~1e-14 relative: R within 1e-13."""
    monkeypatch.setenv("PROM_TCURVE", "0")   # the windowed path (k_order); transmission curves: test_gpu_tcurve.py
    from prometheus_amd import configs
    cfg = configs.get(name) if name in ("C3", "C4") else json.loads(str(load("transit_" + name)["config"]))
    tr = _product_transit(cfg)
    monkeypatch.setenv("PROM_SPECIES_MERGE", merge)
    monkeypatch.setenv("PROM_SIGMA_ROWS", "0")
    R_b = tr.sumOverChords(devices=[0])
    monkeypatch.setenv("PROM_SIGMA_ROWS", "1")
    monkeypatch.setenv("PROM_SIG_POLY", "0")
    R_a = tr.sumOverChords(devices=[0])
    monkeypatch.setenv("PROM_SIG_POLY", "1")
    R_p = tr.sumOverChords(devices=[0])
    print(name, "merge", merge, "exp10 rows max rel diff %.3e" % rel(R_a, R_b), "poly rows %.3e" % rel(R_p, R_b))
    assert np.array_equal(R_a, R_b)
    assert rel(R_p, R_b) < 1e-13
    assert np.array_equal(np.isnan(R_p), np.isnan(R_b))


# ---- SERPENS gridded density, tidally heated moon, setup-file harness (fixtures: oracle/gen_golden.py)
def test_serpens_golden(dev, tmp_path):
    """SerpensExosphere through the CLI loader (prometheus.py:100-105): the histogram grid sampled on the
    device (PROM_DENSITY_GRIDDED) inside the fused path, and the standalone sampler on the reference's
    scalar calculateNumberDensity calls."""
    from prometheus_amd import configs, setupfile
    d = load("serpens")
    path = configs.synthetic_serpens_particles(str(tmp_path / "serpens.txt"), n=int(d["particles_n"]),
                                               seed=int(d["particles_seed"]))
    cfg = json.loads(str(d["config"]))
    cfg["Scenarios"]["serpens"]["serpensPath"] = path
    tr = setupfile.build_transit(cfg)
    assert np.array_equal(tr.wavelength, d["wavelength"])
    sc = tr.atmosphere.densityDistributionList[0]
    for i in range(len(d["kat_phi"])):
        n = sc.calculateNumberDensity(d["kat_x"], d["kat_phi"][i], d["kat_rho"][i], 0.)
        assert rel(n, d["kat_n"][i]) < 1e-13
    # batched chords (the reference's batch call fails; each row equals its scalar call)
    nb = sc.calculateNumberDensity(d["kat_x"], d["kat_phi"], d["kat_rho"], np.zeros(len(d["kat_phi"])))
    assert rel(nb, d["kat_n"]) < 1e-13
    R = tr.sumOverChords()
    assert rel(R, d["R"]) < R_TOL
    assert np.min(d["R"]) < 0.99   # the cloud absorbs


def test_tidal_golden(dev, tmp_path):
    """TidallyHeatedMoon (host plugin, tabulated onto the device) against the reference's R."""
    from prometheus_amd import configs, gasProperties as gp, celestialBodies as bodies, geometryHandler as geom
    d = load("tidal")
    path = configs.synthetic_mdot(str(tmp_path / "mdot.txt"), n=int(d["mdot_n"]), seed=int(d["mdot_seed"]))
    cfg = json.loads(str(d["config"]))
    g, arch, T = cfg["Grids"], cfg["Architecture"], configs.TIDAL
    planet = bodies.AvailablePlanets().findPlanet(arch["planetName"])
    moon = bodies.Moon(arch["starting_orbphase_moon"], arch["R_moon"], arch["a_moon"], planet)
    sgrid = geom.Grid(g["x_midpoint"], g["x_border"], int(g["x_steps"]), g["upper_rho"], int(g["rho_steps"]),
                      int(g["phi_steps"]), g["orbphase_border"], int(g["orbphase_steps"]))
    wgrid = gp.WavelengthGrid(g["lower_w"], g["upper_w"], g["widthHighRes"], g["resolutionLow"], g["resolutionHigh"])
    sc = gp.TidallyHeatedMoon(T["q"], moon)
    sc.addSourceRateFunction(path, T["tau"], T["mass"])
    sc.addConstituent("NaI", T["sigma_v"])
    sc.constituents[-1].addLookupFunctionToConstituent(wgrid)
    tr = gp.Transit(gp.Atmosphere([sc], True), wgrid, sgrid)
    tr.addWavelength()
    assert np.array_equal(tr.wavelength, d["wavelength"])
    assert rel(tr.sumOverChords(), d["R"]) < R_TOL


@pytest.mark.parametrize("name", ["C1", "C2h"])
def test_setup_harness_golden(dev, name, tmp_path):
    """setup JSON -> output file through `python -m prometheus_amd.setupfile` (prometheus.py:56-156): same
    header, phase row and wavelength column bitwise, R within the north-star tolerance."""
    from prometheus_amd import setupfile
    d = load("harness")
    (tmp_path / "setupFiles").mkdir()
    (tmp_path / "setupFiles" / (name + ".txt")).write_text(str(d["setup_" + name]))
    setupfile.run(name, path=str(tmp_path))
    ours = (tmp_path / "output" / (name + ".txt")).read_text()
    ref = str(d["output_" + name])
    head = [l for l in ref.splitlines() if l.startswith("#")]
    assert [l for l in ours.splitlines() if l.startswith("#")] == head
    a = np.loadtxt(str(tmp_path / "output" / (name + ".txt")))
    b = np.loadtxt(ref.splitlines())
    assert a.shape == b.shape
    assert np.array_equal(a[0, 1:], b[0, 1:]) and np.array_equal(a[1:, 0], b[1:, 0])
    assert rel(a[1:, 1:], b[1:, 1:]) < R_TOL


def test_band_lightcurve_reference_script(dev):
    """Transit.bandLightcurve (k_band_stats over R in HBM) against the light curve computed by the
    reference's own mainRetrieval.py section (lightcurve.npz): the light curve is pinned, not only restated."""
    d = load("lightcurve")
    tr = _product_transit(json.loads(str(d["config"])))
    lc, R = tr.bandLightcurve(return_spectrum=True)
    assert rel(R, d["R"]) < R_TOL
    assert rel(lc, d["lightcurve"]) < R_TOL
