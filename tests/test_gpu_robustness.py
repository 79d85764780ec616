"""GPU robustness: paths the golden-vector tests do not reach -- table lifetime, pipelined runs of every
column path, phases with more active chords than the sorted-window limit, the multi-chunk memory
budget and density profiles whose n_0 does not bound them.  Each result is checked against the CPU
oracle (tolerance 1e-10 relative, the north star) or bitwise against the product's own reference run.
"""
import gc
import json
import os

import numpy as np
import pytest

from oracle import prom_oracle as O

pytestmark = pytest.mark.gpu

R_TOL = 1e-10
G = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
    r[(a == b)] = 0.0
    return float(np.max(r)) if r.size else 0.0


@pytest.fixture(scope="module")
def dev():
    from prometheus_amd import _native
    return _native.get_device(0)


def _oracle_R(cfg, wav):
    scen, dop, grids = O.from_setup(cfg)
    return O.transit_depth(scen, dop, grids, wav, O.build_tables(scen, grids))


def test_table_free_keeps_memory_flat(dev):
    """Building and dropping lookup tables (a retrieval loop rebuilding its atmosphere, n_interp_log
    per call) leaves the context's table count and device bytes flat: ids are freed and reused."""
    from prometheus_amd import gasProperties as gp
    x = np.linspace(5.8e-5, 5.9e-5, 20000)
    y = -20. + np.sin(x * 1e7)
    gc.collect()
    with dev.lock:
        dev._drain_frees()
        base = dev.table_count()
    for i in range(30):
        t = gp.LookupTable(x, y + i, 1e-50)
        with dev.lock:
            tid = t.table_id(dev)
            assert dev.table_lookup(tid, x[:5]).shape == (5,)
        del t
        gc.collect()
        out = gp.n_interp_log(x[:7], x, y, 1e-50)
        assert rel(out, 10 ** np.interp(x[:7], x, y) - 1e-50) < 1e-13
    with dev.lock:
        dev._drain_frees()
        after = dev.table_count()
    # one live table at most: x, y (8 B per node), the bucket directory (4 B per bucket, 4 n + 1 buckets)
    # and the interval records (32 B per node)
    one = 8 * 20000 * 2 + 4 * (4 * 20000 + 1) + 32 * 20000
    assert after[0] <= base[0] + 1 and after[2] <= base[2] + one


def test_freed_table_invalidates_problem(dev):
    """A transit problem that reads a freed table cannot run (PROM_E_STATE), instead of reading freed
    device memory; setting it again works."""
    from prometheus_amd import _native
    d = np.load(os.path.join(G, "transit_C1.npz"))
    from prometheus_amd import setupfile
    tr = setupfile.build_transit(json.loads(str(d["config"])))
    host = tr._host_inputs()
    with dev.lock:
        dev.transit_set(tr._problem(dev, host, 0, len(tr.wavelength), 0.0))
        dev.transit_run()
        con = tr.atmosphere.densityDistributionList[0].constituents[0]
        tid = con.lookupFunction.table_id(dev)
        dev.table_free(tid)
        con.lookupFunction._ids.pop(dev.device)
        with pytest.raises(_native.NativeError, match="STATE|prom_transit_set"):
            dev.transit_run()
    R = tr.sumOverChords(devices=[0])   # re-uploads the table and sets the problem again
    assert rel(R, d["R"]) < R_TOL


@pytest.mark.parametrize("x_steps", [30, 80])
def test_pipelined_runs_bitwise(dev, x_steps):
    """Eight back-to-back runs without synchronisation (the pipelined fast path rotates slots and
    streams; the generic column path of n_x > 64 runs on one slot): the last run's R is bitwise the
    R of a single synchronised run."""
    from prometheus_amd import configs, setupfile
    cfg = configs.reduced(configs.get("C2"), orbphase_steps=3, lower_w=5886e-8, upper_w=5900e-8,
                          res_low=5e-9, res_high=1e-10)
    cfg["Grids"]["x_steps"] = x_steps
    tr = setupfile.build_transit(cfg)
    R1 = tr.sumOverChords(devices=[0])
    host = tr._host_inputs()
    with dev.lock:
        dev.transit_set(tr._problem(dev, host, 0, len(tr.wavelength), 0.0))
        for _ in range(8):
            dev.transit_run()
        R8 = dev.transit_result()
    assert np.array_equal(R1, R8)
    assert rel(R1, _oracle_R(cfg, tr.wavelength)) < R_TOL


@pytest.mark.parametrize("stagger", ["0", "1"])
def test_pipelined_doppler_runs_bitwise(dev, stagger, monkeypatch):
    """Orbital Doppler shift (sigma rows per phase), eight back-to-back runs over the pipeline slots, with
    and without the staggered kernel order (PROM_SIG_STAGGER=1: odd slots queue k_sigma_rows after
    k_order): every run's R is bitwise the R of a single synchronised run."""
    from prometheus_amd import setupfile
    d = np.load(os.path.join(G, "transit_C3r.npz"))
    tr = setupfile.build_transit(json.loads(str(d["config"])))
    R1 = tr.sumOverChords(devices=[0])
    monkeypatch.setenv("PROM_SIG_STAGGER", stagger)
    host = tr._host_inputs()
    with dev.lock:
        dev.transit_set(tr._problem(dev, host, 0, len(tr.wavelength), 0.0))
        for _ in range(8):
            dev.transit_run()
        R8 = dev.transit_result()
        dev.transit_run()
        dev.synchronize()
        R9 = dev.transit_result()
    assert np.array_equal(R1, R8) and np.array_equal(R1, R9)
    assert rel(R1, d["R"]) < R_TOL


def test_more_active_chords_than_window_limit(dev):
    """100 x 50 = 5,000 chords per phase, nearly all active (power law q = 6): more than the sorted
    window limit (4,096), so the phases take the unsorted compaction and the heavy tau units; checked
    against the oracle."""
    from prometheus_amd import configs, setupfile
    cfg = configs.reduced(configs.get("C3"), phi_steps=100, rho_steps=50, orbphase_steps=2,
                          lower_w=5886e-8, upper_w=5900e-8, res_low=2e-9, res_high=2e-10)
    cfg["Scenarios"]["powerLaw"]["P_0"] = 1e-1
    tr = setupfile.build_transit(cfg)
    R = tr.sumOverChords(devices=[0])
    st = tr.last_stats[-1]
    print("active %d of %d chord-phases, records %d" % (st["active_chords"], 2 * 5000, st["tau_records"]))
    assert st["active_chords"] > 2 * 4096
    assert st["tau_records"] == st["active_chords"]   # unsorted phases: no merging
    assert rel(R, _oracle_R(cfg, tr.wavelength)) < R_TOL


def test_multi_chunk_memory_budget(dev):
    """A tiny max_memory_gb processes each shard in several 4,096-wavelength chunks (the analogue of
    memoryHandler.py:55-66's batching): R and the band light curve are bitwise the one-chunk results."""
    from prometheus_amd import setupfile
    d = np.load(os.path.join(G, "transit_C2r.npz"))
    tr = setupfile.build_transit(json.loads(str(d["config"])))
    R1 = tr.sumOverChords(devices=[0])
    n1 = len(tr.last_stats)
    Rc = tr.sumOverChords(devices=[0], max_memory_gb=1e-9)
    nc = len(tr.last_stats)
    assert n1 == 1 and nc >= 2 and nc == -(-len(tr.wavelength) // 4096)
    assert np.array_equal(R1, Rc)
    lc1 = tr.bandLightcurve(devices=[0])
    lcc = tr.bandLightcurve(devices=[0], max_memory_gb=1e-9)
    assert rel(lcc, lc1) < 1e-14
    assert rel(Rc, d["R"]) < R_TOL


@pytest.mark.parametrize("q", [-0.5, 1.5])
def test_unbounded_density_profile_disables_windows(dev, q):
    """A power law growing outwards (q < 0) is not bounded by n_0: windows are switched off (variant
    1x) and R still matches the oracle; q >= 0 keeps them (variant 2x/3x)."""
    from prometheus_amd import configs, setupfile
    cfg = configs.reduced(configs.get("C3"), orbphase_steps=2, lower_w=5886e-8, upper_w=5900e-8,
                          res_low=5e-9, res_high=5e-10)
    cfg["Scenarios"]["powerLaw"]["q_esc"] = q
    cfg["Scenarios"]["powerLaw"]["P_0"] = 1e-6
    tr = setupfile.build_transit(cfg)
    R = tr.sumOverChords(devices=[0])
    st = tr.last_stats[-1]
    print("q", q, "variant", st["tau_kernel_variant"])
    assert (st["tau_kernel_variant"] // 10 == 1) == (q < 0)
    assert rel(R, _oracle_R(cfg, tr.wavelength)) < R_TOL


def test_band_lightcurve_array_centres(dev):
    """bandLightcurve accepts a numpy array of line centres (no truth-value ambiguity)."""
    from prometheus_amd import setupfile, lightcurve as lc
    d = np.load(os.path.join(G, "transit_C2r.npz"))
    tr = setupfile.build_transit(json.loads(str(d["config"])))
    a = tr.bandLightcurve(devices=[0])
    b = tr.bandLightcurve(line_centers=np.array([lc.NA_D2, lc.NA_D1]), devices=[0])
    assert np.array_equal(a, b)


def test_pinned_result_arrays(dev):
    """sumOverChords returns R in page-locked memory from the library's pool (one DMA, prom_host_alloc):
    the values are bitwise those copied into ordinary memory, a dropped array's buffer is reused, and past
    the pool's cap (PROM_PINNED_CAP_MB) no new buffer is handed out (sumOverChords then uses ordinary
    memory)."""
    from prometheus_amd import _native, configs, setupfile
    cfg = configs.reduced(configs.get("C2"), orbphase_steps=3, lower_w=5886e-8, upper_w=5900e-8,
                          res_low=5e-9, res_high=1e-10)
    tr = setupfile.build_transit(cfg)
    R1 = tr.sumOverChords(devices=[0])
    assert isinstance(R1.base, _native._PinnedBuffer) and R1.flags.writeable and R1.flags.c_contiguous
    with dev.lock:
        Rp = dev.transit_result(out=np.empty_like(R1))   # pageable: staged path
    assert np.array_equal(R1, Rp)
    del R1
    gc.collect()
    R2 = tr.sumOverChords(devices=[0])
    addr = R2.__array_interface__["data"][0]
    del R2
    gc.collect()
    R2 = tr.sumOverChords(devices=[0])
    assert R2.__array_interface__["data"][0] == addr    # the freed buffer came back
    view = R2[1:]
    del R2
    gc.collect()
    assert np.array_equal(view, Rp[1:])                  # a view keeps its buffer alive
    old = os.environ.get("PROM_PINNED_CAP_MB")
    os.environ["PROM_PINNED_CAP_MB"] = "0"
    try:
        # a cached buffer is still handed out (it adds no pinned bytes); a new one is refused
        assert _native.host_array((8192, 8191)) is None   # larger than any cached buffer
    finally:
        if old is None:
            del os.environ["PROM_PINNED_CAP_MB"]
        else:
            os.environ["PROM_PINNED_CAP_MB"] = old
    assert rel(Rp, _oracle_R(cfg, tr.wavelength)) < R_TOL


def test_sigma_segments_reused_across_problems(dev):
    """prom_transit_set keeps the Doppler sigma segments of the previous problem when the wavelengths, tables
    and Doppler factors are unchanged, and rebuilds them when any of them changes: every run of a problem is
    bitwise its first run, and each problem matches the oracle."""
    from prometheus_amd import configs, setupfile
    cfg = configs.reduced(configs.get("C4"), orbphase_steps=3, lower_w=5886e-8, upper_w=5900e-8,
                          res_low=5e-9, res_high=1e-10)
    tr = setupfile.build_transit(cfg)
    cfg2 = json.loads(json.dumps(cfg))
    cfg2["Grids"]["orbphase_border"] = 0.07    # other phases: other Doppler factors, same wavelengths
    tr2 = setupfile.build_transit(cfg2)
    assert np.array_equal(tr.wavelength, tr2.wavelength)
    seq = [tr, tr, tr2, tr, tr2, tr2]
    got = [t.sumOverChords(devices=[0]).copy() for t in seq]
    for i in (1, 3):
        assert np.array_equal(got[i], got[0])
    for i in (4, 5):
        assert np.array_equal(got[i], got[2])
    assert not np.array_equal(got[0], got[2])
    assert rel(got[0], _oracle_R(cfg, tr.wavelength)) < R_TOL
    assert rel(got[2], _oracle_R(cfg2, tr2.wavelength)) < R_TOL


def test_failed_set_does_not_commit_sigma_segments(dev):
    """A prom_transit_set that builds new Doppler sigma segments and then fails (here: a stellar table with
    a non-zero offset, rejected after the segments are built) must not leave its segment key behind: the
    same problem without the star rebuilds the segments instead of reusing ones that never reached the
    device, and matches the oracle (prom_api.hip seg_key_valid)."""
    from prometheus_amd import configs, setupfile, _native
    cfg = configs.reduced(configs.get("C4"), orbphase_steps=3, lower_w=5886e-8, upper_w=5900e-8,
                          res_low=5e-9, res_high=1e-10)
    tr = setupfile.build_transit(cfg)
    R_a = tr.sumOverChords(devices=[0]).copy()
    cfg2 = json.loads(json.dumps(cfg))
    cfg2["Grids"]["orbphase_border"] = 0.07    # other Doppler factors: the segments are rebuilt
    tr2 = setupfile.build_transit(cfg2)
    host = tr2._host_inputs()
    con = host["scenarios"][0]["dist"].constituents[0].lookupFunction   # offset 1e-50: not a star table
    n_pr = len(host["y"])
    host_bad = dict(host, stellar={"rho": np.ones(n_pr), "clv": np.ones(n_pr), "shift": np.ones(n_pr), "table": con})
    with dev.lock:
        with pytest.raises(_native.NativeError):
            dev.transit_set(tr2._problem(dev, host_bad, 0, len(tr2.wavelength), 0.0))
    R_c = tr2.sumOverChords(devices=[0])
    assert rel(R_c, _oracle_R(cfg2, tr2.wavelength)) < R_TOL
    assert rel(R_a, _oracle_R(cfg, tr.wavelength)) < R_TOL


def test_molecular_zero_cross_sections(dev):
    """A molecular table that is zero over half its wavenumbers (log10(0 + offset) = the floor): where every
    in-table sample's cross-section is zero, the reference's tau is exactly 0 (R: the unblocked share of the disk
    flux); the table-exp path subtracts the offset per sample (n_abs (10^v - offset)), so tau there is at most
    ~1e-14 offset n_abs dx and e^-tau is 1.0: R within 1e-14 of the oracle there, and within R_TOL everywhere."""
    from prometheus_amd import configs
    from prometheus_amd import gasProperties as gp
    from prometheus_amd import setupfile
    tab = O.synthetic_molecular_table(n_nu=2001)
    tab["xsecarr"][:, :, :1000] = 0.0          # nu < 7500 cm^-1: lambda > 1.333 um
    gp.register_molecular_table("H2O", tab)
    try:
        cfg = configs.fixture_configs()["C5r"]
        tr = setupfile.build_transit(cfg)
        R = tr.sumOverChords(devices=[0])
        scen, dop, grids = O.from_setup(cfg, {"H2O": tab})
        Ro = O.transit_depth(scen, dop, grids, tr.wavelength, O.build_tables(scen, grids))
        zero = tr.wavelength > 1.0 / 7490.0   # (the bins from 7497.5 cm^-1 up interpolate to nonzero values)
        assert zero.any() and (~zero).any()
        # tau = 0 there: the reference's R is the unblocked share of the disk flux, ours to rounding
        assert float(np.max(np.abs(R[:, zero] - Ro[:, zero]))) < 1e-14
        assert rel(R, Ro) < R_TOL
    finally:
        gp.register_molecular_table("H2O", O.synthetic_molecular_table(n_nu=2001))
