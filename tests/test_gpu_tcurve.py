"""The transmission-curve path (prom_tcurve.hip), the default for one effective absorber: R(o, w) =
T_o(Y(o, w)) with T_o from a per-phase tail polynomial and per-octave Chebyshev tables.

Against the reference's golden vectors at the north-star tolerance (1e-10 relative), and against the exact
chord sums of the validation path (PROM_OPT_NO_WINDOW: every chord, ocml-free table exp, no windows) within
the path's own bound (a few 1e-16 per unit weight plus rounding; tested at 1e-13 absolute).  The exact
per-point fallback above a truncated table (PROM_TC_LG) and the non-finite-column path are exercised too.
"""
import json
import os

import numpy as np
import pytest

from oracle import prom_oracle as O

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(__file__), "golden")
R_TOL = 1e-10
TC_TOL = 1e-13


def load(name):
    return np.load(os.path.join(G, name + ".npz"))


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
    from prometheus_amd import setupfile
    return setupfile.build_transit(cfg)


ATOMIC = ["C1", "C2r", "C3r", "C4r", "exomoon"]


@pytest.mark.parametrize("name", ATOMIC)
def test_tcurve_default_and_golden(dev, name):
    d = load("transit_" + name)
    tr = _transit(json.loads(str(d["config"])))
    tr.collect_stats = True
    R = tr.sumOverChords(devices=[0])
    st = tr.last_stats[-1]
    assert st["tau_kernel_variant"] in (81, 91), st   # the transmission-curve path took the run
    assert rel(R, d["R"]) < R_TOL


@pytest.mark.parametrize("name", ATOMIC)
def test_tcurve_matches_exact_sums(dev, name):
    from prometheus_amd import _native
    d = load("transit_" + name)
    tr = _transit(json.loads(str(d["config"])))
    R = tr.sumOverChords(devices=[0])
    R_ex = tr.sumOverChords(devices=[0], options=_native.OPT_NO_WINDOW | _native.OPT_NO_MERGE)
    err = float(np.max(np.abs(R - R_ex)))
    print("%s: |R_tc - R_exact| max %.3e" % (name, err))
    assert err < TC_TOL


@pytest.mark.parametrize("name", ["C2r", "C3r", "exomoon"])
def test_tcurve_truncated_table_exact_fallback(dev, name, monkeypatch):
    """PROM_TC_LG=1: one octave of table; every point above it takes the exact per-point sum."""
    d = load("transit_" + name)
    cfg = json.loads(str(d["config"]))
    R = _transit(cfg).sumOverChords(devices=[0])
    monkeypatch.setenv("PROM_TC_LG", "1")
    R1 = _transit(cfg).sumOverChords(devices=[0])
    assert float(np.max(np.abs(R - R1))) < TC_TOL
    assert rel(R1, d["R"]) < R_TOL


@pytest.mark.parametrize("name", ["C2r", "C4r"])
def test_tcurve_against_previous_path(dev, name, monkeypatch):
    """PROM_TCURVE=0 keeps the windowed path (k_order, fused rows / k_tau_p); both are within their bounds."""
    d = load("transit_" + name)
    cfg = json.loads(str(d["config"]))
    R = _transit(cfg).sumOverChords(devices=[0])
    monkeypatch.setenv("PROM_TCURVE", "0")
    tr = _transit(cfg)
    tr.collect_stats = True
    R0 = tr.sumOverChords(devices=[0])
    assert tr.last_stats[-1]["tau_kernel_variant"] not in (81, 91)
    assert float(np.max(np.abs(R - R0))) < 1e-13


def test_tcurve_sharding_bitwise(dev):
    """Wavelength shards (256-aligned) and phase subsets give bitwise the full problem's R."""
    d = load("transit_C3r")
    tr = _transit(json.loads(str(d["config"])))
    R = tr.sumOverChords(devices=[0])
    R3 = tr.sumOverChords(devices=[0, 0, 0])
    assert np.array_equal(R, R3)


def test_tcurve_stats_count_table_exps(dev):
    d = load("transit_C3r")
    tr = _transit(json.loads(str(d["config"])))
    tr.collect_stats = True
    tr.sumOverChords(devices=[0])
    st = tr.last_stats[-1]
    # 16 Chebyshev nodes per table octave, every active chord at each
    assert st["exp_evals"] > 0 and st["exp_evals"] % 16 == 0


@pytest.mark.parametrize("name", ["C3r", "C4r", "exomoon"])
def test_tcurve_exp10_lookups(dev, name, monkeypatch):
    """PROM_SIG_POLY=0: the transmission-curve kernel with numpy.interp + exp10 lookups (the variant coarse
    tables take) against the polynomial lookups (1e-13) and the reference."""
    d = load("transit_" + name)
    cfg = json.loads(str(d["config"]))
    R = _transit(cfg).sumOverChords(devices=[0])
    monkeypatch.setenv("PROM_SIG_POLY", "0")
    tr = _transit(cfg)
    tr.collect_stats = True
    R0 = tr.sumOverChords(devices=[0])
    assert tr.last_stats[-1]["tau_kernel_variant"] in (81, 91)
    assert rel(R0, R) < 1e-13
    assert rel(R0, d["R"]) < R_TOL


def test_bucket_directories(dev, monkeypatch, capfd):
    """Oversize sigma blocks without a linear guess look their brackets up in per-block bucket directories
    (SigSeg kind & 32, verified on the host at every target): exomoon has some (PROM_DEBUG's count) and its R
    agrees with the directory-free lookups (PROM_SEG_DIR=0) within the path's bound and with the golden R."""
    d = load("transit_exomoon")
    cfg = json.loads(str(d["config"]))
    monkeypatch.setenv("PROM_DEBUG", "1")
    R = _transit(cfg).sumOverChords(devices=[0])
    err = capfd.readouterr().err
    n_dir = [int(l.split(":")[1].split(",")[0]) for l in err.splitlines() if "bucket directories" in l]
    assert n_dir and n_dir[-1] > 0
    monkeypatch.setenv("PROM_SEG_DIR", "0")
    R0 = _transit(cfg).sumOverChords(devices=[0])
    err = capfd.readouterr().err
    assert any("bucket directories: 0," in l for l in err.splitlines())
    assert float(np.max(np.abs(R - R0))) < TC_TOL
    assert rel(R, d["R"]) < R_TOL


def test_kernel_ms_ids_match_the_path(dev):
    """prom_transit_kernel_ms times each kernel under the id prom_hip.h documents for it: on the transmission-
    curve path k_columns8 (columns), k_tc_build (tc_build) and k_sigma_tc (sigma_tc) and nothing else; on the
    molecular path k_chords (order) and k_tau_mol (tau)."""
    from prometheus_amd import _native, gasProperties as gp
    d = load("transit_C3r")
    tr = _transit(json.loads(str(d["config"])))
    host = tr._host_inputs()
    dv = _native.get_device(0)
    with dv.lock:
        dv.transit_set(tr._problem(dv, host, 0, len(tr.wavelength), 0.0))
        kms = dv.transit_kernel_ms(3)
    assert set(kms) == set(_native.KERNEL_IDS)
    timed = {k for k, v in kms.items() if v is not None}
    assert timed == {"columns", "tc_build", "sigma_tc"}, kms
    gp.register_molecular_table("H2O", O.synthetic_molecular_table(n_nu=2001))
    d = load("transit_C5r")
    tr = _transit(json.loads(str(d["config"])))
    host = tr._host_inputs()
    with dv.lock:
        dv.transit_set(tr._problem(dv, host, 0, len(tr.wavelength), 0.0))
        kms = dv.transit_kernel_ms(2)
    timed = {k for k, v in kms.items() if v is not None}
    assert timed == {"columns", "order", "tau"}, kms
