"""CPU checks of the SERPENS, tidally-heated-moon and setup-harness fixtures (tests/golden/serpens.npz,
tidal.npz, harness.npz, made by oracle/gen_golden.py from the reference itself).

* the oracle's restatements reproduce the reference's numbers bitwise (histogram grid, scalar densities,
  absorber numbers, R);
* the product's host-side set-up (SERPENS histogram, tidal source-rate interpolation, the setup-file
  writer's layout) is bitwise the reference's -- these run without a GPU.
The device halves of the same paths are in tests/test_gpu_parity.py."""
import json
import os

import numpy as np
import pytest

from oracle import prom_oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(G, name + ".npz"))


def serpens_setup(tmp_path):
    """The fixture's config with its particle file regenerated from the recorded seed."""
    from prometheus_amd import configs
    d = load("serpens")
    path = configs.synthetic_serpens_particles(str(tmp_path / "serpens.txt"), n=int(d["particles_n"]),
                                               seed=int(d["particles_seed"]))
    cfg = json.loads(str(d["config"]))
    cfg["Scenarios"]["serpens"]["serpensPath"] = path
    return d, cfg, path


def test_serpens_oracle_grid_and_kats(tmp_path):
    d, cfg, path = serpens_setup(tmp_path)
    N = cfg["Species"]["serpens"]["NaI"]["Nparticles"]
    xp, yp, zp, vals = O.serpens_grid(path, N, cfg["Grids"])
    for a, k in ((xp, "grid_x"), (yp, "grid_y"), (zp, "grid_z"), (vals, "values")):
        assert np.array_equal(a, d[k]), k
    assert np.array_equal(O.serpens_grid(path, N, cfg["Grids"], 1.5)[3], d["values_smoothed"])
    for i in range(len(d["kat_phi"])):
        n = O.serpens_density((xp, yp, zp, vals), d["kat_x"], d["kat_phi"][i], d["kat_rho"][i])
        assert np.array_equal(n, d["kat_n"][i])


def test_serpens_oracle_transit(tmp_path):
    d, cfg, _ = serpens_setup(tmp_path)
    wav, orb, R = O.run_setup(cfg)
    assert np.array_equal(wav, d["wavelength"])
    assert np.array_equal(R, d["R"]), np.max(np.abs(R / d["R"] - 1))


def test_serpens_product_histogram(tmp_path):
    """SerpensExosphere.addInterpolatedDensity (host numpy, as the reference) gives the reference's grid."""
    from prometheus_amd import gasProperties as gp, geometryHandler as geom, celestialBodies as bodies
    d, cfg, path = serpens_setup(tmp_path)
    g = cfg["Grids"]
    sgrid = geom.Grid(g["x_midpoint"], g["x_border"], int(g["x_steps"]), g["upper_rho"], int(g["rho_steps"]),
                      int(g["phi_steps"]), g["orbphase_border"], int(g["orbphase_steps"]))
    planet = bodies.AvailablePlanets().findPlanet("WASP-49b")
    for smooth, key in ((0., "values"), (1.5, "values_smoothed")):
        sc = gp.SerpensExosphere(path, cfg["Species"]["serpens"]["NaI"]["Nparticles"], planet, smooth)
        sc.addInterpolatedDensity(sgrid)
        assert np.array_equal(sc.gridValues, d[key])
        for a, k in zip(sc.gridAxes, ("grid_x", "grid_y", "grid_z")):
            assert np.array_equal(a, d[k])
    kind, params, body = sc.densityModel()
    assert body is None and params == [len(d["grid_x"]), len(d["grid_y"]), len(d["grid_z"])]
    # the reference's bounds_error: a point outside the grid is a ValueError naming the dimension
    with pytest.raises(ValueError, match="dimension 1"):
        sc.checkBounds(d["grid_x"][:1], [2. * g["upper_rho"]], [0.])


def tidal_objects(tmp_path):
    from prometheus_amd import configs
    d = load("tidal")
    path = configs.synthetic_mdot(str(tmp_path / "mdot.txt"), n=int(d["mdot_n"]), seed=int(d["mdot_seed"]))
    return d, json.loads(str(d["config"])), path


def test_tidal_oracle(tmp_path):
    from prometheus_amd import configs
    d, cfg, path = tidal_objects(tmp_path)
    T = configs.TIDAL
    scen, dop, grids = O.from_setup(cfg)
    sc = scen[0]
    sc.kind = "tidal"
    sc.params = {"q": T["q"], "source": O.tidal_source(path, T["tau"], T["mass"])}
    sc.constituents = [{"species": "NaI", "chi": 1., "sigma_v": T["sigma_v"]}]
    assert np.array_equal(O.tidal_absorber_number(sc, d["kat_orb"]), d["kat_N"])
    cg = d["kat_chords"]
    assert np.array_equal(O.number_density(sc, d["kat_x"], cg[:, 0], cg[:, 1], cg[:, 2]), d["kat_n"])
    tabs = O.build_tables(scen, grids)
    wav = O.simulation_wavelengths(grids, O.atomic_species(scen))
    assert np.array_equal(wav, d["wavelength"])
    R = O.transit_depth(scen, dop, grids, wav, tabs)
    assert np.array_equal(R, d["R"]), np.max(np.abs(R / d["R"] - 1))


def test_tidal_product_host_plugin(tmp_path):
    """TidallyHeatedMoon's host-side numbers (absorber number, tabulated density) are the reference's."""
    from prometheus_amd import configs, gasProperties as gp, celestialBodies as bodies
    d, cfg, path = tidal_objects(tmp_path)
    arch, T = cfg["Architecture"], configs.TIDAL
    planet = bodies.AvailablePlanets().findPlanet(arch["planetName"])
    moon = bodies.Moon(arch["starting_orbphase_moon"], arch["R_moon"], arch["a_moon"], planet)
    sc = gp.TidallyHeatedMoon(T["q"], moon)
    sc.addSourceRateFunction(path, T["tau"], T["mass"])
    assert np.array_equal(sc.calculateAbsorberNumber(d["kat_orb"]), d["kat_N"])
    cg = d["kat_chords"]
    assert np.array_equal(sc.calculateNumberDensity(d["kat_x"], cg[:, 0], cg[:, 1], cg[:, 2]), d["kat_n"])


@pytest.mark.parametrize("name", ["C1", "C2h"])
def test_harness_oracle_and_writer(name, tmp_path):
    """prometheus.py's output file for a setup JSON: the oracle's R is the reference's (bitwise), and the
    product's writer (setupfile.write_output) lays the same numbers out byte for byte."""
    from prometheus_amd import setupfile
    d = load("harness")
    cfg = json.loads(str(d["setup_" + name]))
    ref_text = str(d["output_" + name])
    wav, orb, R = O.run_setup(cfg)
    out = tmp_path / "out.txt"
    setupfile.write_output(str(out), wav, orb, R)
    assert out.read_text() == ref_text


def test_lightcurve_oracle_matches_reference_script():
    """The oracle's light curve (mainRetrieval.py:73-93 restated) on the reference's R equals the light curve
    the reference's own script section computed (lightcurve.npz)."""
    d = load("lightcurve")
    cfg = json.loads(str(d["config"]))
    planet = O.load_planet(cfg["Architecture"]["planetName"])
    lc = O.lightcurve(d["R"], d["wavelength"], d["orbphase"], planet)
    assert np.array_equal(lc, d["lightcurve"])


def test_star_table_cache_follows_content():
    """The device copy of an Fstar_function is cached per function object and content: replacing or
    modifying its arrays in place gives a fresh table (no stale spectrum)."""
    from prometheus_amd import gasProperties as gp

    class Fn:
        pass

    fn = Fn()
    fn.x = np.linspace(5e-5, 6e-5, 101)
    fn.y = np.linspace(14.0, 14.5, 101)
    t1 = gp._star_lookup_table(fn)
    assert gp._star_lookup_table(fn) is t1            # unchanged: the cached table
    fn.y[7] += 0.25                                    # in place
    t2 = gp._star_lookup_table(fn)
    assert t2 is not t1 and t2.y[7] == fn.y[7]
    fn.y = fn.y.copy()                                 # replaced, same content: still valid
    assert gp._star_lookup_table(fn) is t2
    fn.x = fn.x * 1.0000001                            # replaced, new content
    assert gp._star_lookup_table(fn) is not t2
