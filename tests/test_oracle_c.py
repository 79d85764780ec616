"""The C restatement of the molecular optical depth (oracle/mol_tau.c, test infrastructure) against the numpy
oracle (prom_oracle.molecular_sigma: scipy's RegularGridInterpolator, gasProperties.py:774-818), which the
golden vectors pin (tests/test_oracle_golden.py).  The C path only makes full-size samples affordable
(tests/test_gpu_fullsize.py C5); it must agree with the numpy oracle to rounding, including the fill value
outside the table (P below 1e-4 clip / above the grid, lambda outside the table) and the grid nodes.
"""
import numpy as np
import pytest

from oracle import prom_oracle as O


@pytest.fixture(scope="module")
def rgi():
    O.build_c()
    return O.molecular_interpolator(O.synthetic_molecular_table(n_p=6, n_t=5, n_nu=401, seed=3))


def test_mol_tau_c_matches_numpy(rgi):
    rng = np.random.default_rng(5)
    Pg, Tg, lg = rgi.grid
    nc, nx = 7, 9
    P = 10 ** rng.uniform(-5, 10, (nc, nx))            # below the 1e-4 clip, inside and above the grid
    P[0, :4] = Pg[:4]                                 # exactly on P nodes
    P[1, 0], P[1, 1] = Pg[0], Pg[-1]                  # the table's P edges
    n = rng.uniform(1e10, 1e20, (nc, nx))
    shifts = 1.0 + rng.uniform(-3e-4, 3e-4, nc)
    wav = np.concatenate([np.linspace(lg[0] * 0.999, lg[-1] * 1.001, 301), lg[:5], lg[-5:]])
    wav[-10:] /= shifts[2]                            # shifted wavelength exactly on nodes for chord 2
    for T in (Tg[0], 0.5 * (Tg[1] + Tg[2]), Tg[-1], Tg[-1] + 1.0):
        tau_np = np.einsum("cx,cxw->cw", n * 0.3, O.molecular_sigma(rgi, P, T, shifts[:, None] * wav[None, :])) * 7.5
        tau_c = np.zeros((nc, len(wav)))
        O.molecular_tau_c(rgi, n * 0.3, P, T, shifts, wav, 7.5, tau_c)
        scale = np.maximum(np.abs(tau_np), 1e-300)
        assert np.max(np.abs(tau_c - tau_np) / scale) < 1e-13, T
        if T > Tg[-1]:
            assert np.all(tau_c == 0.0)


def test_transit_depth_mol_c_matches_numpy():
    """A reduced C5-like molecular transit through both oracle paths."""
    from prometheus_amd import configs
    cfg = configs.get("C5")
    g = dict(cfg["Grids"])
    g.update(phi_steps=6, rho_steps=5, orbphase_steps=3, x_steps=10)
    cfg = dict(cfg, Grids=g)
    scen, dop, grids = O.from_setup(cfg, {"H2O": O.synthetic_molecular_table()})
    tabs = O.build_tables(scen, grids)
    wav = np.linspace(float(g["lower_w"]), float(g["upper_w"]), 23)
    R_np = O.transit_depth(scen, dop, grids, wav, tabs)
    R_c = O.transit_depth(scen, dop, grids, wav, tabs, mol_c=True)
    assert np.max(np.abs(R_c / R_np - 1.0)) < 1e-13
