#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE itself (container-only).

TEST INFRASTRUCTURE.  Imports CrazeXD/Prometheus from /root/reference with stub
modules for the three optional imports that are absent in this image
(``numba`` -> identity ``njit``/``prange = range``, so ``n_interp_log`` runs as the
plain Python loop it is; ``h5py`` -> an in-memory provider of the seeded
synthetic molecular table; ``astropy.io.fits`` -> empty, never called on the
CLI path).  Nothing from the reference is copied: this script only calls it and
stores inputs and outputs as small ``.npz`` fixtures under ``tests/golden/``.

    python oracle/gen_golden.py            # writes tests/golden/*.npz

The GPU box never runs this (the reference does not exist there).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import types

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("PROMETHEUS_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from prometheus_amd import configs  # noqa: E402  (plain setup dicts, no compute)
from oracle.prom_oracle import synthetic_molecular_table  # noqa: E402

# ---------------------------------------------------------------- stubs
_MOLECULAR = {}


class _FakeH5:
    """Stands in for h5py.File(<molecularResources>/<mol>.h5, 'r+') (gasProperties.py:774)."""

    def __init__(self, path, mode="r"):
        name = os.path.basename(path)[:-3]
        self.d = _MOLECULAR[name]

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def __getitem__(self, k):
        return np.asarray(self.d[k])


def _install_stubs():
    sys.dont_write_bytecode = True   # nothing is written under the reference tree
    numba = types.ModuleType("numba")
    numba.njit = lambda *a, **k: (a[0] if a and callable(a[0]) else (lambda f: f))
    numba.prange = range
    h5py = types.ModuleType("h5py")
    h5py.File = _FakeH5
    astropy = types.ModuleType("astropy")
    io = types.ModuleType("astropy.io")
    fits = types.ModuleType("astropy.io.fits")
    astropy.io, io.fits = io, fits
    sys.modules.update({"numba": numba, "h5py": h5py, "astropy": astropy,
                        "astropy.io": io, "astropy.io.fits": fits})
    sys.path.insert(0, REF)


_install_stubs()
import pythonScripts.celestialBodies as bodies  # noqa: E402
import pythonScripts.constants as const  # noqa: E402
import pythonScripts.gasProperties as gasprop  # noqa: E402
import pythonScripts.geometryHandler as geom  # noqa: E402


def reference_transit(cfg: dict):
    """Build reference objects from a setup dict the way prometheus.py:66-134 does,
    by calling the reference's own classes, and return (transit, scenario list)."""
    arch, scen, spec, g = cfg["Architecture"], cfg["Scenarios"], cfg["Species"], cfg["Grids"]
    planet = bodies.AvailablePlanets().findPlanet(arch["planetName"])
    wgrid = gasprop.WavelengthGrid(g["lower_w"], g["upper_w"], g["widthHighRes"],
                                   g["resolutionLow"], g["resolutionHigh"])
    sgrid = geom.Grid(g["x_midpoint"], g["x_border"], int(g["x_steps"]), g["upper_rho"],
                      int(g["rho_steps"]), int(g["phi_steps"]), g["orbphase_border"],
                      int(g["orbphase_steps"]))
    lst = []
    for key, prm in scen.items():
        if key == "barometric":
            lst.append(gasprop.BarometricAtmosphere(prm["T"], prm["P_0"], prm["mu"], planet))
        elif key == "hydrostatic":
            lst.append(gasprop.HydrostaticAtmosphere(prm["T"], prm["P_0"], prm["mu"], planet))
        elif key == "powerLaw":
            if "P_0" in prm:
                lst.append(gasprop.PowerLawAtmosphere(prm["T"], prm["P_0"], prm["q_esc"], planet))
            else:
                sp0 = list(spec["powerLaw"].keys())[0]
                lst.append(gasprop.PowerLawExosphere(spec["powerLaw"][sp0]["Nparticles"],
                                                     prm["q_esc"], planet))
        elif key == "exomoon":
            moon = bodies.Moon(arch["starting_orbphase_moon"], arch["R_moon"], arch["a_moon"], planet)
            sp0 = list(spec["exomoon"].keys())[0]
            lst.append(gasprop.MoonExosphere(spec["exomoon"][sp0]["Nparticles"], prm["q_moon"], moon))
        elif key == "torus":
            sp0 = list(spec["torus"].keys())[0]
            lst.append(gasprop.TorusExosphere(spec["torus"][sp0]["Nparticles"], prm["a_torus"],
                                              prm["v_ej"], planet))
    names = const.AvailableSpecies().listSpeciesNames()
    for i, (key, prm) in enumerate(scen.items()):
        for sp, ab in spec[key].items():
            if "T" in prm:
                if sp in names:
                    lst[i].addConstituent(sp, ab["chi"])
                    lst[i].constituents[-1].addLookupFunctionToConstituent(wgrid)
                else:
                    lst[i].addMolecularConstituent(sp, ab["chi"])
                    lst[i].constituents[-1].addLookupFunctionToConstituent()
            else:
                if sp in names:
                    lst[i].addConstituent(sp, ab["sigma_v"])
                    lst[i].constituents[-1].addLookupFunctionToConstituent(wgrid)
                else:
                    lst[i].addMolecularConstituent(sp, ab["T"])
                    lst[i].constituents[-1].addLookupFunctionToConstituent()
    atmos = gasprop.Atmosphere(lst, cfg["Fundamentals"]["DopplerOrbitalMotion"])
    tr = gasprop.Transit(atmos, wgrid, sgrid)
    tr.addWavelength()
    return tr, lst, sgrid


def _save(name, **arrays):
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, "%.1f kB" % (os.path.getsize(path) / 1e3))


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def gen_transits():
    _MOLECULAR["H2O"] = synthetic_molecular_table(n_nu=2001)
    for name, cfg in configs.fixture_configs().items():
        tr, lst, sgrid = reference_transit(cfg)
        R = tr.sumOverChords(max_memory_gb=2.0)
        # a second run with tiny batches exercises the np.add.at branch (gasProperties.py:1254-1256)
        R_small = tr.sumOverChords(max_memory_gb=2e-5)
        tables = {}
        for si, sc in enumerate(lst):
            for ci, c in enumerate(sc.constituents):
                if not c.isMolecule:
                    tables["table_%d_%d_x" % (si, ci)] = c.lookupFunction.x
                    tables["table_%d_%d_y" % (si, ci)] = c.lookupFunction.y
        _save("transit_" + name, R=R, R_small_batches=R_small, wavelength=tr.wavelength,
              orbphase=sgrid.constructOrbphaseAxis(), config=np.array(json.dumps(cfg)), **tables)


def gen_multi():
    """Several density scenarios in one atmosphere, and atoms with a molecule in one scenario
    (configs.multi_fixture_configs; gasProperties.py:906-954, prometheus.py:74-129)."""
    _MOLECULAR[configs.VIS_MOLECULE] = configs.visible_molecular_table()
    for name, cfg in configs.multi_fixture_configs().items():
        tr, lst, sgrid = reference_transit(cfg)
        R = tr.sumOverChords(max_memory_gb=2.0)
        # chords are batched so that every batch holds every phase's chords only partly (np.add.at branch)
        R_small = tr.sumOverChords(max_memory_gb=2e-3)
        _save("multi_" + name, R=R, R_small_batches=R_small, wavelength=tr.wavelength,
              orbphase=sgrid.constructOrbphaseAxis(), config=np.array(json.dumps(cfg)))


def gen_stars():
    """Stellar-spectrum fixtures (gasProperties.py:1180-1219): CLV + RM rotation + a synthetic
    spectrum installed as the reference's interp1d Fstar_function (celestialBodies.py:223-235)."""
    from scipy.interpolate import interp1d
    from oracle.prom_oracle import synthetic_star_spectrum
    cfgs = configs.star_fixture_configs()
    for name, (cname, star) in configs.STAR_FIXTURES.items():
        cfg = cfgs[cname]
        tr, lst, sgrid = reference_transit(cfg)
        hs = tr.planet.hostStar
        g = cfg["Grids"]
        x, F = synthetic_star_spectrum(g["lower_w"], g["upper_w"])
        hs.addCLVparameters(star["u1"], star["u2"])
        hs.addRMparameters(star["vsini"], star["phi_rot"])
        hs.Fstar_function = interp1d(x, np.log10(F))
        try:
            R = tr.sumOverChords(max_memory_gb=2.0)
        finally:
            hs.addCLVparameters(0., 0.)
            hs.addRMparameters(0., 0.)
            hs.Fstar_function = None
        _save(name, R=R, wavelength=tr.wavelength, orbphase=sgrid.constructOrbphaseAxis(),
              config=np.array(json.dumps(cfg)), star=np.array(json.dumps(star)),
              fstar_sha=np.array(_sha(np.concatenate([x, np.log10(F)]))))


def gen_star_methods():
    """Star.round_to_grid / calculateRM / getFstar / getFstarIntegrated (celestialBodies.py:113-333) of the
    reference, on WASP-49's star with CLV coefficients, a synthetic spectrum installed as the reference's
    interp1d Fstar_function, and a small disk grid: the closed form (vsini = 0) and the rotating branch."""
    from scipy.interpolate import interp1d
    from oracle.prom_oracle import synthetic_star_spectrum
    planet = bodies.AvailablePlanets().findPlanet("WASP-49b")
    st = planet.hostStar
    lo, hi = 5886e-8, 5896e-8
    x, F = synthetic_star_spectrum(lo, hi)
    wav = np.linspace(lo, hi, 301)
    grid = geom.Grid(planet.a, 5. * planet.R, 10, 0.8 * st.R, 6, 7, 0.1, 3)
    pts = np.array([[0.3, 0.2 * st.R], [2.1, 0.55 * st.R], [4.0, 0.9 * st.R], [5.9, 0.05 * st.R]])
    out = {"wavelength": wav, "spec_x": x, "spec_logF": np.log10(F), "points": pts, "R_star": np.array(st.R),
           "grid": np.array([grid.x_midpoint, grid.x_border, grid.x_steps, grid.rho_border, grid.rho_steps,
                             grid.phi_steps, grid.orbphase_border, grid.orbphase_steps])}
    cases = {"static": (0.31, 0.22, 0.0, 0.0), "rot": (0.31, 0.22, 5e6, 0.4), "rot_noclv": (0.0, 0.0, 3e6, -1.1)}
    for name, (u1, u2, vsini, phi_rot) in cases.items():
        st.addCLVparameters(u1, u2)
        st.addRMparameters(vsini, phi_rot)
        st.Fstar_function = interp1d(x, np.log10(F))
        try:
            FI, FU = st.getFstarIntegrated(wav, grid)
            out[name + "_integrated"] = FI
            out[name + "_upper"] = FU
            out[name + "_getFstar"] = np.array([st.getFstar(p[0], p[1], wav) for p in pts])
            if vsini != 0.0:
                out[name + "_calculateRM"] = np.array([st.calculateRM(p[0], p[1], wav) for p in pts])
            out[name + "_params"] = np.array([u1, u2, vsini, phi_rot])
        finally:
            st.addCLVparameters(0., 0.)
            st.addRMparameters(0., 0.)
            st.Fstar_function = None
    # round_to_grid on getSpectrum's PHOENIX parameter grids (celestialBodies.py:146-156), ties included
    T_grid = np.concatenate((np.arange(2300, 7100, 100), np.arange(7200, 12200, 200)))
    log_g_grid = np.arange(0, 6.5, 0.5)
    Z_grid = np.concatenate((np.arange(-4, -1, 1), np.arange(-1.5, 1.5, 0.5)))
    alpha_grid = np.arange(0, 1.6, 0.2) - 0.2
    vals = {"T": [2000., 5600., 5650., 7150., 7300., 12500., st.T_eff], "log_g": [-1., 4.25, 4.3, 7.],
            "Z": [-5., -2.5, -1.25, 0.1, 0.25, 2.], "alpha": [-1., 0.1, 0.5, 2.]}
    for key, g in (("T", T_grid), ("log_g", log_g_grid), ("Z", Z_grid), ("alpha", alpha_grid)):
        out["rtg_%s_grid" % key] = g.astype(np.float64)
        out["rtg_%s_values" % key] = np.array(vals[key], dtype=np.float64)
        out["rtg_%s_out" % key] = np.array([bodies.Star.round_to_grid(g, v) for v in vals[key]], dtype=np.float64)
    try:
        st.Fstar_function = interp1d(x, np.log10(F))
        st.addRMparameters(5e6, 0.)
        st.calculateRM(0.0, 0.5 * st.R, np.array([x[0] * 0.9]))
        out["rm_out_of_range_raises"] = np.array(False)
    except ValueError:
        out["rm_out_of_range_raises"] = np.array(True)
    finally:
        st.addRMparameters(0., 0.)
        st.Fstar_function = None
    _save("star_methods", **out)


def gen_wavelength_grids():
    """Full-size lambda grids C1..C5 (hash + samples; C1 stored whole)."""
    out = {}
    for name in ("C1", "C2", "C3", "C4", "C5"):
        cfg = configs.get(name)
        g = cfg["Grids"]
        wg = gasprop.WavelengthGrid(g["lower_w"], g["upper_w"], g["widthHighRes"],
                                    g["resolutionLow"], g["resolutionHigh"])
        planet = bodies.AvailablePlanets().findPlanet("WASP-49b")
        dummies = []
        for key, prm in cfg["Scenarios"].items():
            d = gasprop.BarometricAtmosphere(1000., 1., 1., planet)   # only .constituents is read
            d.constituents = []
            for sp in cfg["Species"][key]:
                if sp in const.AvailableSpecies().listSpeciesNames():
                    d.constituents.append(gasprop.AtmosphericConstituent(
                        const.AvailableSpecies().findSpecies(sp), 1., 1e5))
                else:
                    d.constituents.append(gasprop.MolecularConstituent(sp, 1.))
            dummies.append(d)
        w = wg.constructWavelengthGrid(dummies)
        idx = np.unique(np.linspace(0, len(w) - 1, 257).astype(np.int64))
        out[name + "_n"] = np.int64(len(w))
        out[name + "_sha256"] = np.array(_sha(w))
        out[name + "_idx"] = idx
        out[name + "_samples"] = w[idx]
        if name == "C1":
            out["C1_full"] = w
        out[name + "_config"] = np.array(json.dumps(cfg))
    _save("wavelength_grids", **out)


def gen_tables():
    """Refined log-sigma tables (gasProperties.py:694-715) for several species/temperatures."""
    out = {}
    cases = [("NaI", 5888e-8, 5900e-8, 3000.), ("KI", 7655e-8, 7705e-8, 1500.),
             ("CaII", 3925e-8, 3975e-8, 5000.), ("MgI", 5160e-8, 5190e-8, 2000.),
             ("NaI", 3290e-8, 3310e-8, 800.), ("MgI", 2845e-8, 2860e-8, 2500.)]
    for i, (sp, lo, hi, T) in enumerate(cases):
        wg = gasprop.WavelengthGrid(lo, hi, 2e-8, 5e-9, 2e-10)
        species = const.AvailableSpecies().findSpecies(sp)
        c = gasprop.AtmosphericConstituent(species, 1., np.sqrt(T * const.k_B / species.mass))
        lf = c.constructLookupFunction(wg)
        lines = c.getLineParameters(np.array([lf.x.min(), lf.x.max()]))
        out["case%d_x" % i] = lf.x
        out["case%d_y" % i] = lf.y
        out["case%d_meta" % i] = np.array(json.dumps({"species": sp, "lower_w": lo, "upper_w": hi,
                                                      "T": T, "sigma_v": c.sigma_v}))
        out["case%d_lines" % i] = np.stack(lines)
        # sigma on the raw (not refined) simulation grid as well
        w = wg.constructWavelengthGridSingle(c)
        out["case%d_sigma_direct_w" % i] = w
        out["case%d_sigma_direct" % i] = c.calculateVoigtProfile(w)
    _save("cross_sections", **out)


def gen_interp_kats():
    """n_interp_log known answers (gasProperties.py:34-51): clamps, exact nodes, duplicates."""
    rng = np.random.default_rng(7)
    xg = np.sort(rng.uniform(1.0, 2.0, 300))
    xg[100] = xg[99]                     # an exact duplicate node
    xg[200] = np.nextafter(xg[199], 3.)  # a near-duplicate node
    yg = rng.uniform(-30., -15., 300)
    t = np.concatenate([rng.uniform(0.9, 2.1, 2000), xg[::7], [xg[0], xg[-1], xg[99], xg[199],
                                                                0.5, 2.5, np.nextafter(xg[-1], 3.)]])
    out = gasprop.n_interp_log(t, xg, yg, 1e-50)
    _save("interp_kats", t=t, xg=xg, yg=yg, out=out)


def gen_density():
    """calculateNumberDensity of every CLI-reachable scenario at seeded chords (batch mode)."""
    rng = np.random.default_rng(11)
    planet = bodies.AvailablePlanets().findPlanet("WASP-49b")
    Rs, Rp, a = planet.hostStar.R, planet.R, planet.a
    g = geom.Grid(a, 5 * Rp, 30, Rs, 40, 60, 0.1, 8)
    x = g.constructXaxis()
    n = 256
    rho = np.concatenate([rng.uniform(0.0, 0.3 * Rs, n - 16), rng.uniform(0, Rs, 16)])
    phi = rng.uniform(0, 2 * np.pi, n)
    orb = rng.uniform(-0.12, 0.12, n)
    moon = bodies.Moon(0.65 * 2 * np.pi, const.R_Io, 1.44 * Rp, planet)
    models = {
        "barometric": gasprop.BarometricAtmosphere(3000., 1e4, 2.3 * const.amu, planet),
        "hydrostatic": gasprop.HydrostaticAtmosphere(1500., 1e5, 2.3 * const.amu, planet),
        "powerLawAtm": gasprop.PowerLawAtmosphere(3000., 1e-3, 6., planet),
        "powerLawExo": gasprop.PowerLawExosphere(1e33, 4.5, planet),
        "exomoon": gasprop.MoonExosphere(1e32, 3.34, moon),
        "torus": gasprop.TorusExosphere(1e33, 2 * Rp, 5e5, planet),
    }
    out = {"x": x, "phi": phi, "rho": rho, "orb": orb}
    for k, m in models.items():
        out[k] = m.calculateNumberDensity(x, phi, rho, orb)
    out["moon_params"] = np.array([0.65 * 2 * np.pi, const.R_Io, 1.44 * Rp])
    # orbital geometry (celestialBodies.py:370-397, :499-550)
    out["planet_pos"] = np.stack(planet.getPosition(orb))
    out["planet_vlos"] = planet.getLOSvelocity(orb)
    out["moon_pos"] = np.stack(moon.getPosition(orb))
    out["moon_vlos"] = moon.getLOSvelocity(orb)
    out["doppler"] = const.calculateDopplerShift(-out["planet_vlos"])
    _save("density", **out)


def gen_molecular_kat():
    """MolecularConstituent.getSigmaAbs on a small seeded table (gasProperties.py:765-818)."""
    _MOLECULAR["KAT"] = synthetic_molecular_table(n_p=4, n_t=5, n_nu=64, nu_lo=5000., nu_hi=10000.)
    mc = gasprop.MolecularConstituent("KAT", 1.0)
    mc.addLookupFunctionToConstituent()
    rng = np.random.default_rng(3)
    lam = 1. / np.array([10000., 5000.])
    wav = np.sort(rng.uniform(lam[0] * 0.98, lam[1] * 1.02, (3, 40)), axis=1)
    wav[0, 0] = lam[0]
    wav[0, -1] = lam[1]
    P = 10 ** rng.uniform(-6, 9, (3, 7))
    P[1, 0] = 0.0
    sig = mc.getSigmaAbs(P, 1234.5, wav)
    tab = _MOLECULAR["KAT"]
    _save("molecular_kat", P=P, T=np.float64(1234.5), wav=wav, sigma=sig, **{"tab_" + k: v for k, v in tab.items()})


def gen_serpens():
    """SerpensExosphere (gasProperties.py:519-601) on a seeded synthetic particle file: the reference's
    own histogram grid (sigmaSmoothing 0 and 1.5), scalar calculateNumberDensity calls at seeded chords,
    and R of a reduced transit.  The reference's calculateNumberDensity takes one chord at a time (its
    batched call inside getLOSopticalDepth_Batch builds a ragged array and fails, :905 / :598-600), so
    for the transit each batch is evaluated chord by chord with that same scalar method."""
    import tempfile
    tmp = tempfile.mkdtemp(prefix="serpens_golden_")
    path = configs.synthetic_serpens_particles(os.path.join(tmp, "serpens.txt"))
    cfg = configs.reduced(configs.serpens(path), orbphase_steps=4)
    g = cfg["Grids"]
    planet = bodies.AvailablePlanets().findPlanet(cfg["Architecture"]["planetName"])
    sgrid = geom.Grid(g["x_midpoint"], g["x_border"], int(g["x_steps"]), g["upper_rho"], int(g["rho_steps"]),
                      int(g["phi_steps"]), g["orbphase_border"], int(g["orbphase_steps"]))
    N = cfg["Species"]["serpens"]["NaI"]["Nparticles"]
    smooth = gasprop.SerpensExosphere(path, N, planet, 1.5)
    smooth.addInterpolatedDensity(sgrid)
    sc = gasprop.SerpensExosphere(path, N, planet, 0.)
    sc.addInterpolatedDensity(sgrid)
    rgi = sc.InterpolatedDensity
    rng = np.random.default_rng(21)
    x = sgrid.constructXaxis()
    kat_phi = rng.uniform(0., 2. * np.pi, 24)
    kat_rho = rng.uniform(0., 0.95 * g["upper_rho"], 24)
    kat_n = np.stack([sc.calculateNumberDensity(x, p_, r_, 0.) for p_, r_ in zip(kat_phi, kat_rho)])
    scalar = sc.calculateNumberDensity

    def batched(xx, phi, rho, orb):
        return np.stack([scalar(xx, p_, r_, o_) for p_, r_, o_ in
                         zip(np.atleast_1d(phi), np.atleast_1d(rho), np.atleast_1d(orb))])

    sc.calculateNumberDensity = batched
    sc.addConstituent("NaI", cfg["Species"]["serpens"]["NaI"]["sigma_v"])
    wgrid = gasprop.WavelengthGrid(g["lower_w"], g["upper_w"], g["widthHighRes"], g["resolutionLow"],
                                   g["resolutionHigh"])
    sc.constituents[-1].addLookupFunctionToConstituent(wgrid)
    tr = gasprop.Transit(gasprop.Atmosphere([sc], cfg["Fundamentals"]["DopplerOrbitalMotion"]), wgrid, sgrid)
    tr.addWavelength()
    R = tr.sumOverChords(max_memory_gb=2.0)
    cfg["Scenarios"]["serpens"]["serpensPath"] = "<particle file>"
    _save("serpens", R=R, wavelength=tr.wavelength, orbphase=sgrid.constructOrbphaseAxis(),
          config=np.array(json.dumps(cfg)), grid_x=rgi.grid[0], grid_y=rgi.grid[1], grid_z=rgi.grid[2],
          values=rgi.values, values_smoothed=smooth.InterpolatedDensity.values, kat_x=x, kat_phi=kat_phi,
          kat_rho=kat_rho, kat_n=kat_n, particles_n=np.int64(60000), particles_seed=np.int64(11))


def gen_tidal():
    """TidallyHeatedMoon (gasProperties.py:377-461) on a seeded synthetic M_dot file: absorber numbers
    at seeded phases, batched densities and R of a reduced exomoon-architecture transit."""
    import tempfile
    tmp = tempfile.mkdtemp(prefix="tidal_golden_")
    path = configs.synthetic_mdot(os.path.join(tmp, "mdot.txt"))
    cfg = configs.reduced(configs.exomoon(), orbphase_steps=4)
    g, arch, T = cfg["Grids"], cfg["Architecture"], configs.TIDAL
    planet = bodies.AvailablePlanets().findPlanet(arch["planetName"])
    moon = bodies.Moon(arch["starting_orbphase_moon"], arch["R_moon"], arch["a_moon"], planet)
    sgrid = geom.Grid(g["x_midpoint"], g["x_border"], int(g["x_steps"]), g["upper_rho"], int(g["rho_steps"]),
                      int(g["phi_steps"]), g["orbphase_border"], int(g["orbphase_steps"]))
    wgrid = gasprop.WavelengthGrid(g["lower_w"], g["upper_w"], g["widthHighRes"], g["resolutionLow"],
                                   g["resolutionHigh"])
    sc = gasprop.TidallyHeatedMoon(T["q"], moon)
    sc.addSourceRateFunction(path, T["tau"], T["mass"])
    sc.addConstituent("NaI", T["sigma_v"])
    sc.constituents[-1].addLookupFunctionToConstituent(wgrid)
    rng = np.random.default_rng(8)
    kat_orb = rng.uniform(-3., 3., 32)
    kat_N = sc.calculateAbsorberNumber(kat_orb)
    cg = sgrid.getChordGrid()[:200]
    x = sgrid.constructXaxis()
    kat_n = sc.calculateNumberDensity(x, cg[:, 0], cg[:, 1], cg[:, 2])
    tr = gasprop.Transit(gasprop.Atmosphere([sc], True), wgrid, sgrid)
    tr.addWavelength()
    R = tr.sumOverChords(max_memory_gb=2.0)
    _save("tidal", R=R, wavelength=tr.wavelength, orbphase=sgrid.constructOrbphaseAxis(),
          config=np.array(json.dumps(cfg)), kat_orb=kat_orb, kat_N=kat_N, kat_chords=cg, kat_x=x, kat_n=kat_n,
          mdot_n=np.int64(40), mdot_seed=np.int64(5))


def gen_harness():
    """The reference's own CLI harness (prometheus.py:23-165) end to end: setup JSON -> output file.
    prometheus.py reads <PATH>/setupFiles/<name>.txt and writes <PATH>/output/<name>.txt with PATH the
    folder enclosing the checkout; it is executed here (its source compiled as is, under the name
    __main__) with __file__ pointing into a scratch tree, so PATH is that scratch folder and nothing is
    written under /root/reference."""
    import contextlib
    import io
    import tempfile
    src_path = os.path.join(REF, "prometheus.py")
    with open(src_path) as fh:
        code = compile(fh.read(), src_path, "exec")
    out = {}
    for name, cfg in (("C1", configs.c1()),
                      ("C2h", configs.reduced(configs.c2(), orbphase_steps=3, res_low=5e-9, res_high=2e-10,
                                              lower_w=5886e-8, upper_w=5900e-8))):
        tmp = tempfile.mkdtemp(prefix="harness_golden_")
        os.makedirs(os.path.join(tmp, "setupFiles"))
        os.makedirs(os.path.join(tmp, "output"))
        text = json.dumps(cfg, indent=2)
        with open(os.path.join(tmp, "setupFiles", name + ".txt"), "w") as fh:
            fh.write(text)
        argv = sys.argv
        sys.argv = ["prometheus.py", name]
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                exec(code, {"__name__": "__main__", "__file__": os.path.join(tmp, "Prometheus", "prometheus.py")})
        finally:
            sys.argv = argv
        with open(os.path.join(tmp, "output", name + ".txt")) as fh:
            out["output_" + name] = np.array(fh.read())
        out["setup_" + name] = np.array(text)
    _save("harness", **out)


def gen_lightcurve():
    """mainRetrieval.py's light-curve extraction (:73-93), executed from the reference's own source text:
    the section from `filterBandwidth = ...` to `lightcurve = np.array(lightcurve)` runs with the
    reference's planet, constants and an R the reference computed (the exomoon fixture's problem).  The
    script as a whole cannot run here (its source-rate file is a path on the author's machine)."""
    with open(os.path.join(REF, "mainRetrieval.py")) as fh:
        text = fh.read()
    a = text.index("filterBandwidth = ")
    b = text.index("lightcurve = np.array(lightcurve)") + len("lightcurve = np.array(lightcurve)")
    code = compile(text[a:b], os.path.join(REF, "mainRetrieval.py"), "exec")
    cfg = configs.fixture_configs()["exomoon"]
    tr, lst, sgrid = reference_transit(cfg)
    R = tr.sumOverChords(max_memory_gb=2.0)
    planet = bodies.AvailablePlanets().findPlanet(cfg["Architecture"]["planetName"])
    g = {"np": np, "const": const, "W49b": planet, "R": R, "wavelength": tr.wavelength,
         "orbphase": sgrid.constructOrbphaseAxis()}
    exec(code, g)
    _save("lightcurve", R=R, wavelength=tr.wavelength, orbphase=g["orbphase"], lightcurve=g["lightcurve"],
          config=np.array(json.dumps(cfg)))


if __name__ == "__main__":
    which = sys.argv[1:] or ["interp", "tables", "density", "grids", "molecular", "transits", "stars",
                             "star_methods", "serpens", "tidal", "harness", "lightcurve", "multi"]
    if "multi" in which:
        gen_multi()
    if "interp" in which:
        gen_interp_kats()
    if "tables" in which:
        gen_tables()
    if "density" in which:
        gen_density()
    if "grids" in which:
        gen_wavelength_grids()
    if "molecular" in which:
        gen_molecular_kat()
    if "transits" in which:
        gen_transits()
    if "stars" in which:
        gen_stars()
    if "star_methods" in which:
        gen_star_methods()
    if "serpens" in which:
        gen_serpens()
    if "tidal" in which:
        gen_tidal()
    if "harness" in which:
        gen_harness()
    if "lightcurve" in which:
        gen_lightcurve()
