"""Host side of the setup-file path (prometheus.py:56-156 equivalent) on the CPU: output layout,
CLI behaviour, wavelength nodes, and the loud failure without a GPU."""
import json
import os

import numpy as np
import pytest

from prometheus_amd import configs, gasProperties as gp, setupfile


def test_output_layout_matches_reference_format(tmp_path):
    # prometheus.py:149-156: row 0 = (NaN, orbital phases / 2 pi); then (wavelength, R[:, w]) per row
    wav = np.array([5.889e-5, 5.890e-5, 5.891e-5])
    orb = np.array([-0.1, 0.0, 0.1])
    R = np.arange(9, dtype=float).reshape(3, 3) / 10.
    f = tmp_path / "out.txt"
    setupfile.write_output(str(f), wav, orb, R)
    lines = f.read_text().splitlines()
    assert lines[0] == "# Prometheus output file."
    assert lines[1] == "# First row: Orbital phases [1]"
    data = np.loadtxt(f)
    assert data.shape == (4, 4)
    assert np.isnan(data[0, 0])
    np.testing.assert_array_equal(data[0, 1:], orb / (2. * np.pi))
    np.testing.assert_array_equal(data[1:, 0], wav)
    np.testing.assert_array_equal(data[1:, 1:], R.T)


def test_cli_help_and_setup_wizard_is_out_of_scope(capsys):
    assert setupfile.main(["--help"]) == 0
    assert setupfile.main(["setup"]) == 2


@pytest.mark.parametrize("name", ["C1", "C2", "C3", "C4"])
def test_wavelength_nodes_equal_the_oracle(name):
    from oracle import prom_oracle as O
    cfg = configs.get(name)
    g = cfg["Grids"]
    scen, dop, grids = O.from_setup(cfg)
    ref = O.simulation_wavelengths(grids, O.atomic_species(scen))
    wg = gp.WavelengthGrid(g["lower_w"], g["upper_w"], g["widthHighRes"], g["resolutionLow"], g["resolutionHigh"])
    lines = []
    for sp in O.atomic_species(scen):
        lines.extend(O.line_parameters(sp, g["lower_w"], g["upper_w"])[0])
    assert np.array_equal(wg.arangeWavelengthGrid(lines), ref)


def test_run_without_gpu_fails_loudly(tmp_path, monkeypatch):
    from prometheus_amd import _native
    if _native.device_count() > 0:
        pytest.skip("a GPU is visible")
    (tmp_path / "setupFiles").mkdir()
    (tmp_path / "setupFiles" / "c1.txt").write_text(json.dumps(configs.get("C1")))
    with pytest.raises(_native.NativeUnavailable):
        setupfile.run("c1", path=str(tmp_path))
    assert not (tmp_path / "output").exists()


def test_lightcurve_host_logic():
    """Band windows and the shard combination of the device partials (sum, count, max) reproduce the
    oracle's light curve (mainRetrieval.py:76-93) on a golden R; partials formed here with numpy."""
    import json
    import os
    import numpy as np
    from oracle import prom_oracle as O
    from prometheus_amd import lightcurve as lc
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "transit_exomoon.npz"))
    cfg = json.loads(str(d["config"]))
    R, wav, orb = d["R"], d["wavelength"], d["orbphase"]
    scen, _, _ = O.from_setup(cfg)
    ref = O.lightcurve(R, wav, orb, scen[0].planet)
    from prometheus_amd import celestialBodies as bodies
    planet = bodies.AvailablePlanets().findPlanet(cfg["Architecture"]["planetName"])
    bounds = lc.band_bounds(lc.planet_shifts(planet, orb))
    acc = lc.BandAccumulator(len(orb))
    for a, b in ((0, 700), (700, 1500), (1500, len(wav))):          # three "shards"
        w = wav[a:b]
        sel = np.zeros((len(orb), b - a), dtype=bool)
        for k in range(bounds.shape[1]):
            sel |= (w[None, :] >= bounds[:, k, 0:1]) & (w[None, :] <= bounds[:, k, 1:2])
        acc.add((R[:, a:b] * sel).sum(axis=1), sel.sum(axis=1), R[:, a:b].max(axis=1))
    got = acc.lightcurve()
    assert np.all(acc.count > 0)
    assert np.max(np.abs(got / ref - 1)) < 1e-13
