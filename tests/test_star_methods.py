"""Star.round_to_grid / calculateRM / getFstar / getFstarIntegrated (celestialBodies.py:113-333) against the
reference's own outputs (tests/golden/star_methods.npz, oracle/gen_golden.py gen_star_methods): the
closed form and the per-point methods on the host (CPU tests), the rotating disk integral on the GPU
(prom_star_disk_flux) and in the oracle restatement."""
import os

import numpy as np
import pytest

from oracle import prom_oracle as O

G = os.path.join(os.path.dirname(__file__), "golden", "star_methods.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(G)


def _star(gold, case):
    from prometheus_amd import celestialBodies as cb, geometryHandler as geom
    planet = cb.AvailablePlanets().findPlanet("WASP-49b")
    st = planet.hostStar
    assert st.R == float(gold["R_star"])
    u1, u2, vsini, phi_rot = gold[case + "_params"]
    st.addCLVparameters(u1, u2)
    st.addRMparameters(vsini, phi_rot)
    st.addFstarSpectrum(gold["spec_x"], 10. ** gold["spec_logF"])
    st.Fstar_function.y = np.ascontiguousarray(gold["spec_logF"])   # the reference's exact log10 F
    g = gold["grid"]
    grid = geom.Grid(g[0], g[1], int(g[2]), g[3], int(g[4]), int(g[5]), g[6], int(g[7]))
    return st, grid


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b) / np.abs(b)))


def test_round_to_grid(gold):
    from prometheus_amd.celestialBodies import Star
    for key in ("T", "log_g", "Z", "alpha"):
        got = [Star.round_to_grid(gold["rtg_%s_grid" % key], v) for v in gold["rtg_%s_values" % key]]
        assert np.array_equal(np.array(got, dtype=np.float64), gold["rtg_%s_out" % key]), key


@pytest.mark.parametrize("case", ["static", "rot", "rot_noclv"])
def test_getFstar_and_calculateRM(gold, case):
    st, _ = _star(gold, case)
    wav = gold["wavelength"]
    for i, (phi, rho) in enumerate(gold["points"]):
        assert rel(st.getFstar(phi, rho, wav), gold[case + "_getFstar"][i]) < 1e-14
        if case != "static":
            assert rel(st.calculateRM(phi, rho, wav), gold[case + "_calculateRM"][i]) < 1e-14


def test_getFstarIntegrated_closed_form(gold):
    st, grid = _star(gold, "static")
    FI, FU = st.getFstarIntegrated(gold["wavelength"], grid)
    assert np.array_equal(FI, gold["static_integrated"])
    assert np.array_equal(FU, gold["static_upper"])


def test_calculateRM_out_of_range_raises(gold):
    st, _ = _star(gold, "rot")
    assert bool(gold["rm_out_of_range_raises"])
    with pytest.raises(ValueError):
        st.calculateRM(0.0, 0.5 * st.R, np.array([gold["spec_x"][0] * 0.9]))


@pytest.mark.parametrize("case", ["rot", "rot_noclv"])
def test_oracle_disk_flux_pinned(gold, case):
    """The oracle's restatement of the rotating branch against the reference's output."""
    st, grid = _star(gold, case)
    u1, u2, vsini, phi_rot = gold[case + "_params"]
    got = O.star_disk_flux(gold["spec_x"], gold["spec_logF"], st.R, u1, u2, vsini, phi_rot, grid.constructPhiAxis(),
                           grid.constructRhoAxis(), grid.getDeltaPhi(), grid.getDeltaRho(), gold["wavelength"])
    assert rel(got, gold[case + "_integrated"]) < 1e-14


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["rot", "rot_noclv"])
def test_getFstarIntegrated_rotating_gpu(gold, case):
    """The rotating disk integral on the GPU (prom_star_disk_flux) against the reference's output; an
    out-of-range target is an error, as the reference's interp1d raises."""
    st, grid = _star(gold, case)
    FI, FU = st.getFstarIntegrated(gold["wavelength"], grid, device=0)
    assert rel(FI, gold[case + "_integrated"]) < 1e-13
    assert np.array_equal(FU, gold[case + "_upper"])
    from prometheus_amd import _native
    with pytest.raises(_native.NativeError):
        st.getFstarIntegrated(np.array([gold["spec_x"][0] * 0.9]), grid, device=0)
