"""Named problem configurations in the reference's setup-file schema.

The reference reads a JSON "setup file" with five sections (written by
``pythonScripts/setup.py:554-581``, read by ``prometheus.py:56-134``); every
value is already in cgs.  The presets below are the BASELINE.json configs
C1..C5 plus reduced variants used for golden fixtures and
parity tests.  They are plain dicts so the same object feeds this package's
loader, the CPU oracle and the reference itself (fixture generator).
"""
from __future__ import annotations

import copy
import csv
import os

_RES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resources")

# cgs constants needed to express grids relative to the system (constants.py:19-26)
_R_J = 7.1492e9
_AU = 1.496e13
_R_SUN = 6.96e10
_KMS = 1e5
_AMU = 1.661 * 10 ** (-24)
_ANG = 1e-8


def _system(name="WASP-49b"):
    """(a, R_p, R_star) in cm from the bundled catalogue (celestialBodies.py:597-638)."""
    stars = {}
    with open(os.path.join(_RES, "stars.csv"), newline="") as fh:
        for row in csv.DictReader(fh):
            stars[row["name"]] = float(row["R_sun"]) * _R_SUN
    with open(os.path.join(_RES, "planets.csv"), newline="") as fh:
        for row in csv.DictReader(fh):
            if row["name"] == name:
                return (float(row["a_AU"]) * _AU, float(row["R_J"]) * _R_J, stars[row["hostStar"]])
    raise KeyError(name)


def _grids(lower_w, upper_w, res_low, res_high, width=2 * _ANG, x_steps=30, rho_steps=40,
           phi_steps=60, orbphase_border=0.1, orbphase_steps=8, planet="WASP-49b"):
    a, Rp, Rs = _system(planet)
    return {"lower_w": lower_w, "upper_w": upper_w, "widthHighRes": width,
            "resolutionLow": res_low, "resolutionHigh": res_high,
            "x_midpoint": a, "x_border": 5. * Rp, "x_steps": x_steps,
            "phi_steps": phi_steps, "rho_steps": rho_steps, "upper_rho": Rs,
            "orbphase_border": orbphase_border, "orbphase_steps": orbphase_steps}


def _fund(doppler):
    return {"ExomoonSource": False, "DopplerPlanetRotation": False, "CLV_variations": False,
            "RM_effect": False, "DopplerOrbitalMotion": bool(doppler)}


def c1():
    """barometric Na, low-res grid (mainRetrieval.py:28,33), 1 phase: CPU plumbing."""
    return {"Fundamentals": _fund(False),
            "Scenarios": {"barometric": {"T": 3000., "P_0": 1e4, "mu": 2.3 * _AMU}},
            "Architecture": {"planetName": "WASP-49b"},
            "Species": {"barometric": {"NaI": {"chi": 1e-6}}},
            "Grids": _grids(5888e-8, 5900e-8, 5e-9, 2e-10, orbphase_border=0., orbphase_steps=1)}


def c2():
    """barometric Na + K, high-res grid, 8 phases (the bench workload at N=1)."""
    return {"Fundamentals": _fund(False),
            "Scenarios": {"barometric": {"T": 3000., "P_0": 1e4, "mu": 2.3 * _AMU}},
            "Architecture": {"planetName": "WASP-49b"},
            "Species": {"barometric": {"NaI": {"chi": 1e-6}, "KI": {"chi": 1e-6}}},
            "Grids": _grids(5880e-8, 7710e-8, 1e-10, 1e-11)}


def c3():
    """pressure-normalised powerLaw (PowerLawAtmosphere), Na I + Ca II + Mg I, Doppler, 16 phases."""
    return {"Fundamentals": _fund(True),
            "Scenarios": {"powerLaw": {"q_esc": 6., "P_0": 1e-3, "T": 3000.}},
            "Architecture": {"planetName": "WASP-49b"},
            "Species": {"powerLaw": {"NaI": {"chi": 1e-6}, "CaII": {"chi": 1e-6},
                                     "MgI": {"chi": 1e-6}}},
            "Grids": _grids(2800e-8, 6000e-8, 1e-10, 1e-11, orbphase_steps=16)}


def c4():
    """Na torus (N=1e33, a=2 R_p, v_ej=5 km/s, sigma_v=10 km/s), Doppler, 8 phases."""
    _, Rp, _ = _system()
    return {"Fundamentals": _fund(True),
            "Scenarios": {"torus": {"a_torus": 2. * Rp, "v_ej": 5. * _KMS}},
            "Architecture": {"planetName": "WASP-49b"},
            "Species": {"torus": {"NaI": {"sigma_v": 10. * _KMS, "Nparticles": 1e33}}},
            "Grids": _grids(5880e-8, 7710e-8, 1e-10, 1e-11)}


def c4x10():
    """C4 at 10x finer resolution (resLow 0.001 A, resHigh 0.0001 A: ~1.8e6 wavelengths), the
    strong-scaling variant of SURVEY.md 8d/8e."""
    cfg = c4()
    cfg["Grids"]["resolutionLow"] = 1e-11
    cfg["Grids"]["resolutionHigh"] = 1e-12
    return cfg


def c4x10p64():
    """C4x10 at 64 orbital phases (1.87e6 wavelengths x 64 phases = 1.2e8 spectrum points): the strong-scaling
    workload whose one-GPU step (~0.5 ms) amortises the per-run chain a shard repeats."""
    cfg = c4x10()
    cfg["Grids"]["orbphase_steps"] = 64
    return cfg


def c4x10p128():
    """C4x10 at 128 orbital phases (2.4e8 spectrum points; 0.66 ms per one-GPU step in round 6)."""
    cfg = c4x10()
    cfg["Grids"]["orbphase_steps"] = 128
    return cfg


def c4x10p256():
    """C4x10 at 256 orbital phases (4.8e8 spectrum points): the >= 1 ms one-GPU strong-scaling workload of the
    N > 1 bench line (bench.py `strong`), split over the ranks by wavelength."""
    cfg = c4x10()
    cfg["Grids"]["orbphase_steps"] = 256
    return cfg


def c2moon():
    """Two density scenarios at C2 size (190,205 wavelengths x 8 phases x 2,400 chords): barometric Na I + K I and a
    moon exosphere of Na I, orbital Doppler shift on -- the planet's and the moon's Doppler factors, chords blocked by
    the moon.  The optical depths of the scenarios add (gasProperties.py:906-954) and cannot merge into one absorber,
    so the run takes the windowed path (k_order, k_tau_p) rather than the transmission curves."""
    _, Rp, _ = _system()
    return {"Fundamentals": dict(_fund(True), ExomoonSource=True),
            "Scenarios": {"barometric": {"T": 3000., "P_0": 1e4, "mu": 2.3 * _AMU}, "exomoon": {"q_moon": 3.34}},
            "Architecture": {"planetName": "WASP-49b", "R_moon": 1.822e8, "a_moon": 1.44 * Rp,
                             "starting_orbphase_moon": 0.65 * 2. * 3.141592653589793},
            "Species": {"barometric": {"NaI": {"chi": 1e-6}, "KI": {"chi": 1e-6}},
                        "exomoon": {"NaI": {"sigma_v": 10. * _KMS, "Nparticles": 1e32}}},
            "Grids": _grids(5880e-8, 7710e-8, 1e-10, 1e-11)}


def c5():
    """hydrostatic + synthetic H2O table, 1-2 micron at 1e-10 cm (1e6 points), 32 phases."""
    return {"Fundamentals": _fund(False),
            "Scenarios": {"hydrostatic": {"T": 1500., "P_0": 1e5, "mu": 2.3 * _AMU}},
            "Architecture": {"planetName": "WASP-49b"},
            "Species": {"hydrostatic": {"H2O": {"chi": 1e-3}}},
            "Grids": _grids(1.0e-4, 2.0e-4, 1e-10, 1e-11, orbphase_steps=32)}


def exomoon():
    """moon exosphere (exomoon scenario, prometheus.py:89-93), Doppler on."""
    _, Rp, _ = _system()
    cfg = {"Fundamentals": _fund(True),
           "Scenarios": {"exomoon": {"q_moon": 3.34}},
           "Architecture": {"planetName": "WASP-49b", "R_moon": 1.822e8,
                            "a_moon": 1.44 * Rp, "starting_orbphase_moon": 0.65 * 2. * 3.141592653589793},
           "Species": {"exomoon": {"NaI": {"sigma_v": 10. * _KMS, "Nparticles": 1e32}}},
           "Grids": _grids(5880e-8, 5910e-8, 5e-10, 1e-11, orbphase_steps=6)}
    cfg["Fundamentals"]["ExomoonSource"] = True
    return cfg


def synthetic_serpens_particles(path, n=60000, seed=11, planet="WASP-49b"):
    """Seeded stand-in for a SERPENS output file (no SERPENS run or file in this image): one particle
    per row, x y z in metres (SerpensExosphere reads it with np.loadtxt and multiplies by 100), written
    with 17 significant digits so the file reads back bit-exactly.  A Gaussian cloud about the planet at
    orbital phase 0, (a, 0, 0), of 1.2 R_p along x and y and 0.8 R_p along z, with a trailing tail
    towards -y (2/5 of the particles).  Returns path."""
    import numpy as np
    rng = np.random.default_rng(seed)
    a, Rp, _ = _system(planet)
    n_tail = 2 * n // 5
    core = rng.normal(0.0, 1.0, (n - n_tail, 3)) * np.array([1.2 * Rp, 1.2 * Rp, 0.8 * Rp])
    s = rng.uniform(0.0, 1.0, n_tail)
    tail = np.stack([rng.normal(0.0, 0.6 * Rp, n_tail), -s * 6.0 * Rp + rng.normal(0.0, 0.4 * Rp, n_tail),
                     rng.normal(0.0, 0.5 * Rp, n_tail)], axis=1)
    pos = np.concatenate([core, tail]) + np.array([a, 0.0, 0.0])
    np.savetxt(path, pos / 1e2, fmt="%.17g")
    return path


def serpens(path):
    """SERPENS exosphere of Na (prometheus.py:100-105) over the particle file at ``path``, Doppler on."""
    return {"Fundamentals": _fund(True),
            "Scenarios": {"serpens": {"serpensPath": path}},
            "Architecture": {"planetName": "WASP-49b"},
            "Species": {"serpens": {"NaI": {"sigma_v": 10. * _KMS, "Nparticles": 2e32}}},
            "Grids": _grids(5884e-8, 5902e-8, 1e-9, 5e-11, orbphase_steps=4)}


def synthetic_mdot(path, n=40, seed=5):
    """Seeded stand-in for a tidally heated moon's mass-loss-rate file (TidallyHeatedMoon
    .addSourceRateFunction, gasProperties.py:404-424): n values of M_dot [g/s] over half a moon orbit,
    log-normal about 1e4 g/s, written with 17 significant digits.  Returns path."""
    import numpy as np
    rng = np.random.default_rng(seed)
    np.savetxt(path, 1e4 * np.exp(0.8 * rng.standard_normal(n)), fmt="%.17g")
    return path


# the tidally heated moon fixture (not reachable from a setup file: the reference CLI has no scenario
# key for it): the exomoon architecture, q, photoionisation lifetime [s] and absorber mass [g]
TIDAL = {"q": 3.34, "tau": 1.2e4, "mass": 22.99 * _AMU, "sigma_v": 10. * _KMS}


PRESETS = {"C1": c1, "C2": c2, "C3": c3, "C4": c4, "C4x10": c4x10, "C4x10p64": c4x10p64, "C4x10p128": c4x10p128, "C4x10p256": c4x10p256,
           "C5": c5, "C2moon": c2moon, "exomoon": exomoon}


def get(name: str) -> dict:
    return copy.deepcopy(PRESETS[name]())


def reduced(cfg: dict, *, phi_steps=12, rho_steps=20, orbphase_steps=None,
            res_low=None, res_high=None, lower_w=None, upper_w=None) -> dict:
    """A spatially/spectrally reduced copy (golden fixtures and CPU-sized parity tests)."""
    out = copy.deepcopy(cfg)
    g = out["Grids"]
    g["phi_steps"], g["rho_steps"] = phi_steps, rho_steps
    if orbphase_steps is not None:
        g["orbphase_steps"] = orbphase_steps
    for k, v in (("resolutionLow", res_low), ("resolutionHigh", res_high),
                 ("lower_w", lower_w), ("upper_w", upper_w)):
        if v is not None:
            g[k] = v
    return out


def fixture_configs():
    """The reduced problems pinned by golden R vectors (tests/golden/transit_*.npz)."""
    return {
        "C1": c1(),
        "C2r": reduced(c2(), orbphase_steps=4, res_low=5e-9, res_high=1e-10),
        "C3r": reduced(c3(), orbphase_steps=4, res_low=1e-8, res_high=5e-10),
        "C4r": reduced(c4(), orbphase_steps=4, res_low=5e-9, res_high=1e-10),
        "C5r": reduced(c5(), orbphase_steps=3, res_low=2.5e-8),
        "exomoon": reduced(exomoon(), orbphase_steps=4),
    }


# A seeded molecular table over the Na D region (16,900-17,050 cm^-1 = 5,866-5,917 A), so one collisional
# scenario can carry atoms and a molecule whose opacities overlap (prometheus.py:109-119 allows any mix).
VIS_MOLECULE = "TiO"


def visible_molecular_table():
    return synthetic_molecular_table(n_nu=601, nu_lo=16900., nu_hi=17050., seed=1)


def multi_fixture_configs():
    """Atmospheres with several density scenarios, or atoms and a molecule in one scenario, pinned by golden
    R vectors (tests/golden/multi_*.npz).  The reference builds one scenario per ``Scenarios`` key
    (prometheus.py:74-105) and sums their optical depths, each with its own Doppler factor (planet or moon),
    in getLOSopticalDepth_Batch (gasProperties.py:906-954)."""
    _, Rp, _ = _system()
    moon_arch = {"planetName": "WASP-49b", "R_moon": 1.822e8, "a_moon": 1.44 * Rp,
                 "starting_orbphase_moon": 0.65 * 2. * 3.141592653589793}
    baro = {"T": 3000., "P_0": 1e4, "mu": 2.3 * _AMU}
    # (i) barometric Na I + K I and a moon exosphere of Na I, orbital Doppler shift on: two scenarios with
    # the planet's and the moon's Doppler factors, and chords blocked by the moon
    baro_moon = {"Fundamentals": dict(_fund(True), ExomoonSource=True),
                 "Scenarios": {"barometric": dict(baro), "exomoon": {"q_moon": 3.34}},
                 "Architecture": dict(moon_arch),
                 "Species": {"barometric": {"NaI": {"chi": 1e-6}, "KI": {"chi": 1e-6}},
                             "exomoon": {"NaI": {"sigma_v": 10. * _KMS, "Nparticles": 1e32}}},
                 "Grids": _grids(5880e-8, 7710e-8, 5e-9, 1e-10, orbphase_steps=4, phi_steps=12, rho_steps=20)}
    # (ii) hydrostatic Na I + a molecule in one scenario, Doppler on: atoms and a molecule in one tau
    mixed = {"Fundamentals": _fund(True),
             "Scenarios": {"hydrostatic": {"T": 1500., "P_0": 1e5, "mu": 2.3 * _AMU}},
             "Architecture": {"planetName": "WASP-49b"},
             "Species": {"hydrostatic": {"NaI": {"chi": 1e-6}, VIS_MOLECULE: {"chi": 1e-4}}},
             "Grids": _grids(5880e-8, 5910e-8, 1e-9, 5e-11, orbphase_steps=3, phi_steps=12, rho_steps=20)}
    # (iii) power-law atmosphere (pressure-normalised) + a Na torus, Doppler on: one Doppler factor, two
    # absorbers with different columns per chord (thermal and torus sigma_v tables); Mg I has no line in the
    # range (its table is the offset floor everywhere, gasProperties.py:1003-1006)
    plaw_torus = {"Fundamentals": _fund(True),
                  "Scenarios": {"powerLaw": {"q_esc": 6., "P_0": 1e-3, "T": 3000.},
                                "torus": {"a_torus": 2. * Rp, "v_ej": 5. * _KMS}},
                  "Architecture": {"planetName": "WASP-49b"},
                  "Species": {"powerLaw": {"NaI": {"chi": 1e-6}, "CaII": {"chi": 1e-6}, "MgI": {"chi": 1e-6}},
                              "torus": {"NaI": {"sigma_v": 10. * _KMS, "Nparticles": 1e33}}},
                  "Grids": _grids(5000e-8, 5900e-8, 5e-9, 1e-10, orbphase_steps=4, phi_steps=12, rho_steps=20)}
    # (iv) all of it, Doppler off: barometric Na I + molecule, moon exosphere, torus (three scenarios)
    three = {"Fundamentals": dict(_fund(False), ExomoonSource=True),
             "Scenarios": {"barometric": dict(baro), "exomoon": {"q_moon": 3.34},
                           "torus": {"a_torus": 2. * Rp, "v_ej": 5. * _KMS}},
             "Architecture": dict(moon_arch),
             "Species": {"barometric": {"NaI": {"chi": 1e-6}, VIS_MOLECULE: {"chi": 1e-5}},
                         "exomoon": {"NaI": {"sigma_v": 10. * _KMS, "Nparticles": 1e32}},
                         "torus": {"NaI": {"sigma_v": 10. * _KMS, "Nparticles": 1e33}}},
             "Grids": _grids(5884e-8, 5902e-8, 1e-9, 5e-11, orbphase_steps=3, phi_steps=12, rho_steps=20)}
    return {"baro_moon": baro_moon, "mixed_mol": mixed, "plaw_torus": plaw_torus, "three": three}


def synthetic_molecular_table(n_p=22, n_t=27, n_nu=50001, nu_lo=5000., nu_hi=10000., seed=0):
    """Seeded stand-in for an ExoMol/TauREx H2O table (no network, no ExoMol data in this image):
    p [Pa] = logspace(-1, 8), t [K] = linspace(100, 3400), bin_edges [cm^-1] = linspace(nu_lo, nu_hi),
    xsecarr[p][t][nu] = 1e-22 exp(N(0, 1))."""
    import numpy as np
    rng = np.random.default_rng(seed)
    return {"p": np.logspace(-1, 8, n_p), "t": np.linspace(100., 3400., n_t),
            "bin_edges": np.linspace(nu_lo, nu_hi, n_nu),
            "xsecarr": 1e-22 * np.exp(rng.standard_normal((n_p, n_t, n_nu)))}


def synthetic_star_spectrum(lower_w, upper_w, step=1e-10, margin=3e-8, seed=7):
    """Seeded stand-in for a PHOENIX HiRes slice (celestialBodies.py:128-209 fetch it over FTP; no
    network here): x = arange(lower_w - margin, upper_w + margin, step) [cm], F = continuum with a
    10 % slope times one Gaussian absorption line per 2 A (depth 5-90 %, sigma 0.05-0.4 A).
    Returns (x, F); Star.addFstarSpectrum(x, F) installs it."""
    import numpy as np
    rng = np.random.default_rng(seed)
    x = np.arange(lower_w - margin, upper_w + margin, step)
    n_lines = max(4, int((x[-1] - x[0]) / 2e-8))
    centre = rng.uniform(x[0], x[-1], n_lines)
    depth = rng.uniform(0.05, 0.9, n_lines)
    width = rng.uniform(0.05e-8, 0.4e-8, n_lines)
    F = 2e14 * (1. + 0.1 * (x - x[0]) / (x[-1] - x[0]))
    for c, d, w in zip(centre, depth, width):
        a, b = np.searchsorted(x, [c - 8. * w, c + 8. * w])
        F[a:b] *= 1. - d * np.exp(-0.5 * ((x[a:b] - c) / w) ** 2)
    return x, F


# stellar-spectrum fixtures: CLV (mainRetrieval.py:38 coefficients), RM rotation, synthetic spectrum
STAR_FIXTURES = {
    "rm_C1": ("C1", {"u1": 0.34, "u2": 0.28, "vsini": 0.0, "phi_rot": 0.0}),
    "rm_C2r": ("C2rs", {"u1": 0.34, "u2": 0.28, "vsini": 5e6, "phi_rot": 0.4}),
    "rm_exomoon": ("exomoon_s", {"u1": 0.0, "u2": 0.0, "vsini": 3e6, "phi_rot": -1.1}),
}


def star_fixture_configs():
    """Setup dicts of the stellar-spectrum fixtures (tests/golden/rm_*.npz)."""
    return {
        "C1": c1(),
        "C2rs": reduced(c2(), orbphase_steps=4, res_low=5e-9, res_high=1e-10, lower_w=5884e-8, upper_w=5900e-8),
        "exomoon_s": reduced(exomoon(), orbphase_steps=3, res_low=2e-9, res_high=5e-11, lower_w=5886e-8,
                             upper_w=5898e-8),
    }
