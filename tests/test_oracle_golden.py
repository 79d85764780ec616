"""Pin the CPU oracle (oracle/prom_oracle.py) to golden vectors from the reference itself.

Fixtures: tests/golden/*.npz, written by oracle/gen_golden.py, which imports the
reference (CrazeXD/Prometheus) with numba/h5py/astropy stubbed.  CPU only.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import prom_oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(G, name + ".npz"))


def test_interp_log_kats():
    d = load("interp_kats")
    out = O.interp_log(d["t"], d["xg"], d["yg"], 1e-50)
    assert np.array_equal(out, d["out"])


def test_wavelength_grids_bitwise():
    d = load("wavelength_grids")
    for name in ("C1", "C2", "C3", "C4", "C5"):
        cfg = json.loads(str(d[name + "_config"]))
        atoms = [s for sc in cfg["Species"].values() for s in sc if s in O.SPECIES]
        w = O.simulation_wavelengths(cfg["Grids"], atoms)
        assert len(w) == int(d[name + "_n"]), name
        assert hashlib.sha256(w.tobytes()).hexdigest() == str(d[name + "_sha256"]), name
        assert np.array_equal(w[d[name + "_idx"]], d[name + "_samples"])
    assert np.array_equal(O.simulation_wavelengths(json.loads(str(d["C1_config"]))["Grids"], ["NaI"]),
                          d["C1_full"])


def test_refined_tables():
    d = load("cross_sections")
    i = 0
    while "case%d_x" % i in d:
        meta = json.loads(str(d["case%d_meta" % i]))
        grid = {"lower_w": meta["lower_w"], "upper_w": meta["upper_w"], "widthHighRes": 2e-8,
                "resolutionLow": 5e-9, "resolutionHigh": 2e-10}
        sv = O.thermal_sigma_v(meta["T"], meta["species"])
        assert sv == meta["sigma_v"]
        x, y = O.refined_table(grid, meta["species"], sv)
        assert np.array_equal(x, d["case%d_x" % i])
        assert np.array_equal(y, d["case%d_y" % i])
        i += 1
    assert i >= 5


def test_density_plugins():
    d = load("density")
    planet = O.load_planet("WASP-49b")
    x, phi, rho, orb = d["x"], d["phi"], d["rho"], d["orb"]
    m0, mR, ma = d["moon_params"]
    moon = O.Body(R=mR, M=0., a=ma, host=planet, orbphase0=m0)
    amu = O.AMU
    cases = {
        "barometric": O.Scenario("barometric", planet, {"T": 3000., "P_0": 1e4, "mu": 2.3 * amu}),
        "hydrostatic": O.Scenario("hydrostatic", planet, {"T": 1500., "P_0": 1e5, "mu": 2.3 * amu}),
        "powerLawAtm": O.Scenario("powerLawAtm", planet, {"T": 3000., "P_0": 1e-3, "q": 6.}),
        "powerLawExo": O.Scenario("powerLawExo", planet, {"N": 1e33, "q": 4.5}),
        "exomoon": O.Scenario("exomoon", planet, {"N": 1e32, "q": 3.34}, moon=moon),
        "torus": O.Scenario("torus", planet, {"N": 1e33, "a_torus": 2 * planet.R, "v_ej": 5e5}),
    }
    for k, sc in cases.items():
        n = O.number_density(sc, x, phi, rho, orb)
        assert np.array_equal(n, d[k]), k
    assert np.array_equal(np.stack(O.planet_position(planet, orb)), d["planet_pos"])
    assert np.array_equal(O.planet_los_velocity(planet, orb), d["planet_vlos"])
    assert np.array_equal(np.stack(O.moon_position(moon, orb)), d["moon_pos"])
    assert np.array_equal(O.moon_los_velocity(moon, orb), d["moon_vlos"])
    assert np.array_equal(O.doppler_shift(-d["planet_vlos"]), d["doppler"])


def test_molecular_kat():
    d = load("molecular_kat")
    tab = {k[4:]: d[k] for k in d.files if k.startswith("tab_")}
    rgi = O.molecular_interpolator(tab)
    sig = O.molecular_sigma(rgi, d["P"], float(d["T"]), d["wav"])
    assert np.array_equal(sig, d["sigma"])


@pytest.mark.parametrize("name", ["C1", "C2r", "C3r", "C4r", "C5r", "exomoon"])
def test_transit_depth(name):
    d = load("transit_" + name)
    cfg = json.loads(str(d["config"]))
    mol = {"H2O": O.synthetic_molecular_table(n_nu=2001)}
    wav, orb, R = O.run_setup(cfg, mol)
    assert np.array_equal(wav, d["wavelength"])
    assert np.array_equal(orb, d["orbphase"])
    # the reference's two reduction branches are bitwise identical (gasProperties.py:1243-1256)
    assert np.array_equal(d["R"], d["R_small_batches"])
    assert np.array_equal(R, d["R"]), np.max(np.abs(R / d["R"] - 1))


def test_synthetic_table_matches_product_copy():
    from prometheus_amd import configs
    a = O.synthetic_molecular_table(n_nu=101)
    b = configs.synthetic_molecular_table(n_nu=101)
    for k in a:
        assert np.array_equal(a[k], b[k])


@pytest.mark.parametrize("name", ["rm_C1", "rm_C2r", "rm_exomoon"])
def test_stellar_spectrum(name):
    """CLV + Rossiter-McLaughlin rotation + a stellar spectrum (gasProperties.py:1180-1219): the oracle
    reproduces the reference bitwise; the synthetic spectrum is the one the fixture was made with."""
    d = load(name)
    cfg = json.loads(str(d["config"]))
    star = json.loads(str(d["star"]))
    g = cfg["Grids"]
    x, F = O.synthetic_star_spectrum(g["lower_w"], g["upper_w"])
    y = np.log10(F)
    sha = hashlib.sha256(np.ascontiguousarray(np.concatenate([x, y])).tobytes()).hexdigest()
    assert sha == str(d["fstar_sha"])
    wav, orb, R = O.run_setup(cfg, None, star=dict(star, fstar=(x, y)))
    assert np.array_equal(wav, d["wavelength"])
    assert np.array_equal(R, d["R"]), np.max(np.abs(R / d["R"] - 1))


def test_synthetic_star_matches_product_copy():
    from prometheus_amd import configs
    a = O.synthetic_star_spectrum(5886e-8, 5890e-8)
    b = configs.synthetic_star_spectrum(5886e-8, 5890e-8)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("name", ["baro_moon", "mixed_mol", "plaw_torus", "three"])
def test_multi_scenario_transit_depth(name):
    """Several density scenarios (planet and moon Doppler factors) and atoms with a molecule in one
    scenario (gasProperties.py:906-954): the oracle reproduces the reference bitwise."""
    from prometheus_amd import configs
    d = load("multi_" + name)
    cfg = json.loads(str(d["config"]))
    mol = {configs.VIS_MOLECULE: O.synthetic_molecular_table(n_nu=601, nu_lo=16900., nu_hi=17050., seed=1)}
    wav, orb, R = O.run_setup(cfg, mol)
    assert np.array_equal(wav, d["wavelength"])
    assert np.array_equal(orb, d["orbphase"])
    assert np.array_equal(d["R"], d["R_small_batches"])
    assert np.array_equal(R, d["R"]), np.max(np.abs(R / d["R"] - 1))
