"""Full-size parity: every BASELINE.json config at its full size on the HIP path, checked against the
CPU oracle (numpy restatement of gasProperties.py:1160-1258, pinned to the reference's golden vectors
by tests/test_oracle_golden.py) on a seeded sample of wavelengths.  R at one wavelength does not depend
on any other wavelength, so a sampled oracle run is an exact check of those columns of the full-size R,
while the GPU integrates the whole problem: the full chord population (merging, windows, tail moments,
heavy units) and the full grid.

Sizes: C2 190,205 lambda x 8 phases; C3 351,222 x 16 (power law, Na I + Ca II + Mg I,
Doppler); C4 186,604 x 8 (torus, Doppler); C5 1,000,000 x 32 (hydrostatic + H2O, synthetic ExoMol-layout
table); 2,400 chords x 30 samples per phase.  Tolerance: 1e-10 relative (north star).

C5 is checked on 1,000+ wavelengths through the C restatement of the molecular optical depth
(oracle/mol_tau.c, pinned bitwise-close to the numpy oracle by tests/test_oracle_c.py): seeded interior
wavelengths, both ends of the grid (the table's lambda edges coincide with the grid's, so the Doppler-shifted
lookups leave the table there) and the grid wavelengths nearest the table's lambda nodes.
"""
import numpy as np
import pytest

from oracle import prom_oracle as O

pytestmark = pytest.mark.gpu

R_TOL = 1e-10


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    r[(a == b)] = 0.0
    return float(np.max(r)) if r.size else 0.0


def _sample(n_wav, k, seed):
    """k seeded wavelengths plus both grid ends and the centre."""
    rng = np.random.default_rng(seed)
    idx = rng.choice(n_wav, k, replace=False)
    return np.unique(np.concatenate([idx, [0, n_wav // 2, n_wav - 1]]))


# (config, expected shape, sampled wavelengths, seed)
CASES = {
    "C3": ((16, 351222), 400, 13),
    "C4": ((8, 186604), 600, 14),
    "C4x10": ((8, None), 300, 16),    # the 8-GPU strong-scaling workload (~1.9e6 wavelengths)
    "C5": ((32, 1000000), 400, 15),
    "C2moon": ((8, 190205), 400, 17),   # two density scenarios (planet + moon Doppler factors): the windowed path
}


def _c5_sample(wav, table, seed):
    """C5: 400 seeded wavelengths (_sample), 200 over each 1,000-point end of the grid (Doppler-shifted
    lookups cross the table's lambda edges there) and 150 table lambda nodes with both grid neighbours."""
    n = len(wav)
    rng = np.random.default_rng(seed)
    base = _sample(n, 400, seed)
    ends = np.concatenate([np.linspace(0, 999, 200), np.linspace(n - 1000, n - 1, 200)]).astype(np.int64)
    nodes = np.sort(1.0 / np.asarray(table["bin_edges"]))
    nodes = nodes[(nodes > wav[0]) & (nodes < wav[-1])]
    k = np.searchsorted(wav, rng.choice(nodes, 150, replace=False))
    near = np.concatenate([k - 1, k])
    return np.unique(np.concatenate([base, ends, near]))


@pytest.mark.parametrize("name", ["C3", "C4", "C4x10", "C5", "C2moon"])
def test_full_size_config_sampled(name):
    from prometheus_amd import configs, gasProperties as gp, setupfile
    shape, k, seed = CASES[name]
    cfg = configs.get(name)
    mol = None
    if name == "C5":
        mol = {"H2O": O.synthetic_molecular_table()}
        gp.register_molecular_table("H2O", configs.synthetic_molecular_table())
    tr = setupfile.build_transit(cfg)
    R = tr.sumOverChords(devices=[0])
    st = tr.last_stats[-1]
    if shape[1] is None:
        shape = (shape[0], len(tr.wavelength))
    assert R.shape == shape
    if name == "C5":
        idx = _c5_sample(tr.wavelength, mol["H2O"], seed)
        assert len(idx) >= 1000
    else:
        idx = _sample(shape[1], k, seed)
    scen, dop, grids = O.from_setup(cfg, mol)
    Ro = O.transit_depth(scen, dop, grids, tr.wavelength[idx], O.build_tables(scen, grids), mol_c=name == "C5")
    err = rel(R[:, idx], Ro)
    print("%s full size %s: sampled %d wavelengths, max rel err %.3e, stats %s" % (name, shape, len(idx), err, st))
    assert err < R_TOL
    assert np.all(np.isfinite(R)) and np.all((R > 0) & (R <= 1.0 + 1e-12))
    # every chord-phase pair is classified exactly once
    npr = int(cfg["Grids"]["phi_steps"]) * int(cfg["Grids"]["rho_steps"])
    assert st["active_chords"] + st["transparent_chords"] + st["blocked_chords"] == shape[0] * npr


def test_full_size_c3_shards_bitwise():
    """Full C3 split into 2 and 3 wavelength shards (emulated on one GPU) is bitwise the 1-shard R."""
    from prometheus_amd import configs, setupfile
    tr = setupfile.build_transit(configs.get("C3"))
    R1 = tr.sumOverChords(devices=[0])
    assert np.array_equal(R1, tr.sumOverChords(devices=[0, 0]))
    assert np.array_equal(R1, tr.sumOverChords(devices=[0, 0, 0]))


def test_full_size_c4x10_eight_shards_bitwise():
    """The 8-GPU strong-scaling workload C4x10 split into 8 wavelength shards (emulated on one GPU, one host
    thread per shard as on 8 devices) is bitwise the 1-shard R."""
    from prometheus_amd import configs, setupfile
    tr = setupfile.build_transit(configs.get("C4x10"))
    R1 = tr.sumOverChords(devices=[0])
    assert np.array_equal(R1, tr.sumOverChords(devices=[0] * 8))


@pytest.mark.parametrize("name", ["C3", "C4x10", "C4x10p64"])
def test_full_size_tcurve_matches_exact_sums(name):
    """The transmission-curve path (default) against the exact chord sums (every active chord's e^-tau at every
    point, no merging, windows or curves: PROM_OPT_NO_WINDOW | PROM_OPT_NO_MERGE) over the WHOLE full-size grid,
    where the curves' octave count and the column range N_max / N_min are largest.  Bound: the curves' tail and
    Chebyshev truncation (a few 1e-16 per unit weight) plus rounding, tested at 1e-13 absolute; the full-size
    grids carry 5.6e6 (C3), 1.5e7 (C4x10) and 1.2e8 (C4x10p64, 64 phases) points."""
    from prometheus_amd import _native, configs, setupfile
    tr = setupfile.build_transit(configs.get(name))
    tr.collect_stats = True
    R = tr.sumOverChords(devices=[0])
    assert tr.last_stats[-1]["tau_kernel_variant"] // 10 in (8, 9)
    R_ex = tr.sumOverChords(devices=[0], options=_native.OPT_NO_WINDOW | _native.OPT_NO_MERGE)
    err = float(np.max(np.abs(R - R_ex)))
    print("%s full size %s: |R_tc - R_exact| max %.3e" % (name, R.shape, err))
    assert err < 1e-13
