"""Target windows (k_sigma_tw, prometheus_amd/csrc/prom_tw.hip + prom_window.hip): the Doppler-shifted
cross-section lookups of the transmission-curve path grouped by target value instead of by wavelength block.

Every lookup evaluates fl(chi E_k) e^a of numpy's bracket k (gasProperties.py:941-954 via n_interp_log,
:34-51), whatever window, slice kind or pass it falls in, so R must be BITWISE the wavelength-block kernel's
(k_sigma_tc, PROM_TW=0) -- on the golden configs, at full size (C3, C4, C4x10), for wavelength shards and with
the host's window caps forced small (many windows, slices on the global-record and searched paths).  The windows
are the default (PROM_TW=0 switches them off); the tests set PROM_TW=1 explicitly.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _transit(name, reduced=False):
    from prometheus_amd import configs, setupfile
    cfg = configs.get(name)
    if reduced:
        cfg = configs.reduced(cfg)
    return setupfile.build_transit(cfg)


def _windows_line(capfd):
    err = capfd.readouterr().err
    lines = [l for l in err.splitlines() if "target windows" in l]
    return lines[-1] if lines else None


@pytest.mark.parametrize("name", ["C3", "C4", "exomoon"])
def test_windows_bitwise_reduced(name, monkeypatch, capfd):
    monkeypatch.setenv("PROM_DEBUG", "1")
    monkeypatch.setenv("PROM_TW", "1")   # (the default)
    tr = _transit(name, reduced=True)
    R = tr.sumOverChords(devices=[0])
    line = _windows_line(capfd)
    assert line is not None, "the target-window path did not build windows"
    print(name, line)
    monkeypatch.setenv("PROM_TW", "0")
    R0 = tr.sumOverChords(devices=[0])
    assert np.array_equal(R, R0)


@pytest.mark.parametrize("name", ["C3", "C4", "C4x10"])
def test_windows_bitwise_full_size(name, monkeypatch, capfd):
    monkeypatch.setenv("PROM_DEBUG", "1")
    monkeypatch.setenv("PROM_TW", "1")
    tr = _transit(name)
    R = tr.sumOverChords(devices=[0])
    line = _windows_line(capfd)
    assert line is not None
    print(name, R.shape, line)
    monkeypatch.setenv("PROM_TW", "0")
    R0 = tr.sumOverChords(devices=[0])
    assert np.array_equal(R, R0)


def test_windows_shards_bitwise(monkeypatch):
    """Wavelength shards build their own windows; R is bitwise the one-shard R."""
    monkeypatch.setenv("PROM_TW", "1")
    tr = _transit("C4x10")
    R1 = tr.sumOverChords(devices=[0])
    assert np.array_equal(R1, tr.sumOverChords(devices=[0, 0, 0]))


@pytest.mark.parametrize("caps", [("8", "64", "2560"), ("4", "32", "96"), ("256", "8192", "16"),
                                  ("256", "8192", "2560", "0"), ("256", "8192", "2560", "1024", "1"),
                                  ("256", "8192", "2560", "0", "0", "0"),
                                  ("256", "8192", "2560", "1024", "0", "1", "0", "2"),
                                  ("100", "8192", "2560", "0", "0", "1", "64", "2")])
def test_windows_small_caps_bitwise(caps, monkeypatch, capfd):
    """Window caps (wavelengths per row, points per window, LDS doubles[, staged wavelengths, windows grown only while
    their wavelengths fit, exact-guess marks, lane alignment, row pairs]) in a fresh process each: tiny windows, slices
    over the LDS budget (global records, kind 2), a 16-double budget (almost every slice global), wavelengths never
    staged / always staged, the bracket test on every lookup, unaligned windows, two rows per wave with staged and with
    global wavelengths (rows of 100: ragged chunks).  The knobs are read once per process, so each case runs in a
    subprocess."""
    import json
    import os
    import subprocess
    import sys
    env = dict(os.environ, PROM_TW_ROWCAP=caps[0], PROM_TW_PMAX=caps[1], PROM_TW_LDS=caps[2], PROM_DEBUG="1",
               PROM_TW="1")
    for k, v in zip(("PROM_TW_LAMCAP", "PROM_TW_LAMFIT", "PROM_TW_EXACT", "PROM_TW_ALIGN", "PROM_TW_RP"), caps[3:]):
        env[k] = v
    code = (
        "import numpy as np, json, os\n"
        "from prometheus_amd import configs, setupfile\n"
        "tr = setupfile.build_transit(configs.reduced(configs.get('C3')))\n"
        "R = tr.sumOverChords(devices=[0])\n"
        "os.environ['PROM_TW'] = '0'\n"
        "R0 = tr.sumOverChords(devices=[0])\n"
        "print(json.dumps({'eq': bool(np.array_equal(R, R0)), 'shape': list(R.shape)}))\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stderr.splitlines() if "target windows" in l]
    assert lines, p.stderr[-2000:]
    print(caps, lines[0])
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["eq"]


@pytest.mark.parametrize("name", ["C4", "exomoon"])
def test_windows_row_pairs_one_species_bitwise(name):
    """Two rows per wave (PROM_TW_RP=2, read once per process: a subprocess) on one-species problems at their shipped
    sizes (C4 full size: 8 rows; the reduced exomoon golden config): R bitwise the wavelength-block kernel's."""
    import json
    import os
    import subprocess
    import sys
    env = dict(os.environ, PROM_TW_RP="2", PROM_TW="1", PROM_DEBUG="1")
    red = "configs.reduced(configs.get(%r))" % name if name == "exomoon" else "configs.get(%r)" % name
    code = (
        "import numpy as np, json, os\n"
        "from prometheus_amd import configs, setupfile\n"
        "tr = setupfile.build_transit(%s)\n"
        "R = tr.sumOverChords(devices=[0])\n"
        "os.environ['PROM_TW'] = '0'\n"
        "R0 = tr.sumOverChords(devices=[0])\n"
        "print(json.dumps({'eq': bool(np.array_equal(R, R0)), 'shape': list(R.shape)}))\n") % red
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    assert any("target windows" in l for l in p.stderr.splitlines()), p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    print(name, out)
    assert out["eq"]
