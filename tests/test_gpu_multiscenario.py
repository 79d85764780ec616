"""Atmospheres with several density scenarios, and atoms with a molecule in one scenario, on the default
GPU path (no environment overrides) against golden vectors from the reference itself
(tests/golden/multi_*.npz, oracle/gen_golden.py gen_multi; configs.multi_fixture_configs).

The reference sums one optical depth per scenario, each at its own Doppler factor (the planet's or the
moon's line-of-sight velocity), over every constituent, atoms and molecules alike
(gasProperties.py:906-954); the setup harness builds one scenario per Scenarios key (prometheus.py:74-129).
Tolerance: the north-star 1e-10 relative on R.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
R_TOL = 1e-10
NAMES = ["baro_moon", "mixed_mol", "plaw_torus", "three"]


def load(name):
    return np.load(os.path.join(G, "multi_" + name + ".npz"))


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


def _transit(cfg):
    from prometheus_amd import configs
    from prometheus_amd import gasProperties as gp
    from prometheus_amd import setupfile
    gp.register_molecular_table(configs.VIS_MOLECULE, configs.visible_molecular_table())
    return setupfile.build_transit(cfg)


@pytest.mark.parametrize("name", NAMES)
def test_multi_scenario_golden(dev, name):
    d = load(name)
    tr = _transit(json.loads(str(d["config"])))
    assert len(tr.atmosphere.densityDistributionList) >= 1
    assert np.array_equal(tr.wavelength, d["wavelength"])
    tr.collect_stats = True
    R = tr.sumOverChords(devices=[0])
    err = rel(R, d["R"])
    print("%s: max rel err %.3e over %d points, stats %s" % (name, err, R.size, tr.last_stats[-1]))
    assert err < R_TOL


@pytest.mark.parametrize("name", NAMES)
def test_multi_scenario_exact_sums(dev, name):
    """Every chord summed exactly (no merging, windows or tail polynomials) agrees with the default path
    within the approximations' bound and with the reference."""
    from prometheus_amd import _native
    d = load(name)
    tr = _transit(json.loads(str(d["config"])))
    R = tr.sumOverChords(devices=[0])
    R_ex = tr.sumOverChords(devices=[0], options=_native.OPT_NO_WINDOW | _native.OPT_NO_MERGE)
    assert float(np.max(np.abs(R - R_ex))) < 1e-13
    assert rel(R_ex, d["R"]) < R_TOL


@pytest.mark.parametrize("name", NAMES)
def test_multi_scenario_ocml_exp(dev, name):
    from prometheus_amd import _native
    d = load(name)
    tr = _transit(json.loads(str(d["config"])))
    R = tr.sumOverChords(devices=[0], options=_native.OPT_OCML_EXP)
    assert rel(R, d["R"]) < R_TOL


@pytest.mark.parametrize("name", NAMES)
def test_multi_scenario_sharding_bitwise(dev, name):
    """256-aligned wavelength shards (and several chunks) give bitwise the one-shard R."""
    d = load(name)
    tr = _transit(json.loads(str(d["config"])))
    R = tr.sumOverChords(devices=[0])
    assert np.array_equal(R, tr.sumOverChords(devices=[0, 0, 0]))
    assert np.array_equal(R, tr.sumOverChords(devices=[0], max_memory_gb=1e-5))


def test_multi_scenario_pipelined_runs(dev):
    """Consecutive runs of one set rotate over the pipeline slots: every run's R is the same."""
    from prometheus_amd import configs, gasProperties as gp
    d = load("baro_moon")
    tr = _transit(json.loads(str(d["config"])))
    R = [tr.sumOverChords(devices=[0]) for _ in range(6)]
    for r in R[1:]:
        assert np.array_equal(r, R[0])
    assert rel(R[0], d["R"]) < R_TOL
