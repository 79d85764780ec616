"""Setup-file driven runs: the ``prometheus.py`` harness (prometheus.py:23-165) on this package.

    python -m prometheus_amd.setupfile <name> [--max-memory GB] [--devices 0,1,...]

reads ``<PATH>/setupFiles/<name>.txt`` (PATH = parent of the checkout, as in prometheus.py:21;
override with PROMETHEUS_PATH), runs the GPU integrator and writes ``<PATH>/output/<name>.txt`` in
the reference's layout (row 0: NaN then orbital phases / 2 pi; then one row per wavelength:
wavelength [cm], R(phase_0..)).  Differences from the reference harness, all bug fixes that do
not change any result the reference can produce:
  * a number-normalised ``powerLaw`` scenario builds a PowerLawExosphere (the reference crashes
    on ``dict_keys[0]``, prometheus.py:85);
  * the wavelength grid is taken from the Transit object instead of being rebuilt (prometheus.py:142).
"""
from __future__ import annotations

import json
import os
import sys
import time
from typing import Optional, Sequence

import numpy as np

from . import celestialBodies as bodies
from . import constants as const
from . import gasProperties as gasprop
from . import geometryHandler as geom

PATH = os.environ.get("PROMETHEUS_PATH",
                      os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def build_transit(param: dict) -> gasprop.Transit:
    """Objects from a parsed setup file (prometheus.py:59-134)."""
    fund, scen, arch, spec, grids = (param["Fundamentals"], param["Scenarios"], param["Architecture"],
                                     param["Species"], param["Grids"])
    planet = bodies.AvailablePlanets().findPlanet(arch["planetName"])
    if planet is None:
        raise KeyError("planet %r not in the catalogue" % arch["planetName"])
    wgrid = gasprop.WavelengthGrid(grids["lower_w"], grids["upper_w"], grids["widthHighRes"],
                                   grids["resolutionLow"], grids["resolutionHigh"])
    sgrid = geom.Grid(grids["x_midpoint"], grids["x_border"], int(grids["x_steps"]), grids["upper_rho"],
                      int(grids["rho_steps"]), int(grids["phi_steps"]), grids["orbphase_border"],
                      int(grids["orbphase_steps"]))
    models = []
    for key, prm in scen.items():
        first = list(spec.get(key, {}).keys())[:1]
        nparticles = spec[key][first[0]].get("Nparticles") if first else None
        if key == "barometric":
            models.append(gasprop.BarometricAtmosphere(prm["T"], prm["P_0"], prm["mu"], planet))
        elif key == "hydrostatic":
            models.append(gasprop.HydrostaticAtmosphere(prm["T"], prm["P_0"], prm["mu"], planet))
        elif key == "powerLaw":
            if "P_0" in prm:
                models.append(gasprop.PowerLawAtmosphere(prm["T"], prm["P_0"], prm["q_esc"], planet))
            else:
                models.append(gasprop.PowerLawExosphere(nparticles, prm["q_esc"], planet))
        elif key == "exomoon":
            moon = bodies.Moon(arch["starting_orbphase_moon"], arch["R_moon"], arch["a_moon"], planet)
            models.append(gasprop.MoonExosphere(nparticles, prm["q_moon"], moon))
        elif key == "torus":
            models.append(gasprop.TorusExosphere(nparticles, prm["a_torus"], prm["v_ej"], planet))
        elif key == "serpens":
            # sigmaSmoothing hard-coded to 0 as in prometheus.py:103-104
            models.append(gasprop.SerpensExosphere(prm["serpensPath"], nparticles, planet, 0.))
            models[-1].addInterpolatedDensity(sgrid)
        else:
            raise ValueError("unknown scenario %r" % key)
    atoms = const.AvailableSpecies().listSpeciesNames()
    for model, (key, prm) in zip(models, scen.items()):
        collisional = "T" in prm
        for sp, ab in spec[key].items():
            if sp in atoms:
                model.addConstituent(sp, ab["chi"] if collisional else ab["sigma_v"])
                model.constituents[-1].addLookupFunctionToConstituent(wgrid)
            else:
                model.addMolecularConstituent(sp, ab["chi"] if collisional else ab["T"])
                model.constituents[-1].addLookupFunctionToConstituent()
    tr = gasprop.Transit(gasprop.Atmosphere(models, fund["DopplerOrbitalMotion"]), wgrid, sgrid)
    tr.addWavelength()
    return tr


def write_output(path: str, wavelength: np.ndarray, orbphase: np.ndarray, R: np.ndarray) -> None:
    """prometheus.py:149-156."""
    first = np.insert(orbphase / (2. * np.pi), 0, np.nan)
    body = np.vstack((wavelength, R))
    header = ('Prometheus output file.\nFirst row: Orbital phases [1]\n'
              'All other rows: Wavelength [cm] (first column), Transit depth R(orbital phase, wavelength) [1] '
              '(other columns)')
    np.savetxt(path, np.vstack((first, body.T)), header=header)


def run(name: str, max_memory_gb: float = 2.0, devices: Optional[Sequence[int]] = None,
        path: str = PATH) -> np.ndarray:
    t0 = time.time()
    with open(os.path.join(path, "setupFiles", name + ".txt")) as fh:
        param = json.load(fh)
    tr = build_transit(param)
    R = tr.sumOverChords(max_memory_gb=max_memory_gb, devices=devices)
    os.makedirs(os.path.join(path, "output"), exist_ok=True)
    write_output(os.path.join(path, "output", name + ".txt"), tr.wavelength,
                 tr.spatialGrid.constructOrbphaseAxis(), R)
    print("\nPROMETHEUS (MI355X) finished, elapsed time: %.3f s" % (time.time() - t0))
    print("The maximal flux decrease due to atmospheric/exospheric absorption in percent is:",
          np.abs(np.round(100 * (1 - np.min(R)), 5)))
    print("The minimal flux decrease due to atmospheric/exospheric absorption in percent is:",
          np.abs(np.round(100 * (1 - np.max(R)), 5)))
    return R


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    if argv[0] == "setup":
        print("the interactive setup writer (pythonScripts/setup.py) is not part of this build; "
              "write the JSON by hand or use prometheus_amd.configs")
        return 2
    mem = 2.0
    devices = None
    if "--max-memory" in argv:
        try:
            mem = float(argv[argv.index("--max-memory") + 1])
        except (IndexError, ValueError):
            print("Warning: Invalid --max-memory argument. Using default of 2.0 GB")
    if "--devices" in argv:
        devices = [int(v) for v in argv[argv.index("--devices") + 1].split(",")]
    run(argv[0], mem, devices)
    return 0


if __name__ == "__main__":
    sys.exit(main())
