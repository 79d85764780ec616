"""The device Faddeeva / Voigt code (prometheus_amd/csrc/faddeeva.h) compiled for the host with gcc and
checked against mpmath (50 digits) over every region of its piecewise definition, and against scipy's
voigt_profile (the function the reference calls, gasProperties.py:686-690)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = tmp_path_factory.mktemp("fad") / "libfad.so"
    src = os.path.join(REPO, "tests", "helpers", "faddeeva_host.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-o", str(out), src],
                   check=True)
    L = C.CDLL(str(out))
    dp = C.POINTER(C.c_double)
    L.fad_re.argtypes = [C.c_long, dp, dp, dp]
    L.voigt.argtypes = [C.c_long, dp, dp, dp, dp]
    return L


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _fad_re(lib, x, y):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    out = np.empty_like(x)
    lib.fad_re(len(x), _p(x), _p(y), _p(out))
    return out


def _mp_re_w(x, y):
    import mpmath as mp
    mp.mp.dps = 50
    z = mp.mpc(x, y)
    return float(mp.re(mp.exp(-z * z) * mp.erfc(-1j * z)))


def test_faddeeva_regions_against_mpmath(lib):
    rng = np.random.default_rng(7)
    pts = []
    # region A: x < 7, y < 0.25 (Taylor in y); B: x >= 7, y < 1; C: |z| >= 7; D: trapezoid
    pts += list(zip(rng.uniform(0, 7, 60), 10 ** rng.uniform(-12, np.log10(0.25), 60)))
    pts += list(zip(rng.uniform(7, 60, 40), 10 ** rng.uniform(-12, 0, 40)))
    pts += list(zip(rng.uniform(0, 30, 40), rng.uniform(7, 40, 40)))
    pts += list(zip(rng.uniform(0, 6.5, 40), rng.uniform(0.25, 6.5, 40)))
    pts += [(0.0, 0.0), (7.0, 0.25), (6.999999, 0.2499999), (0.0, 7.0), (4.9, 4.9), (1e-300, 1e-300)]
    x = np.array([p[0] for p in pts])
    y = np.array([p[1] for p in pts])
    got = _fad_re(lib, x, y)
    ref = np.array([_mp_re_w(a, b) for a, b in pts])
    rel = np.abs(got - ref) / np.abs(ref)
    assert np.max(rel) < 1e-13, (pts[int(np.argmax(rel))], np.max(rel))
    # symmetry Re w(-x + iy) = Re w(x + iy)
    assert np.array_equal(_fad_re(lib, -x, y), got)


def test_voigt_profile_against_scipy_in_the_line_regime(lib):
    from scipy.special import voigt_profile
    rng = np.random.default_rng(3)
    n = 2000
    # Na D-like parameters (cgs frequencies): sigma ~ 1e9-1e10 Hz, gamma ~ 1e7-1e8 Hz, |x| up to 1e12 Hz
    s = 10 ** rng.uniform(8.5, 10.5, n)
    g = 10 ** rng.uniform(6.5, 8.5, n)
    x = np.sign(rng.uniform(-1, 1, n)) * 10 ** rng.uniform(6, 12, n)
    out = np.empty(n)
    lib.voigt(n, _p(x), _p(s), _p(g), _p(out))
    ref = voigt_profile(x, s, g)
    rel = np.abs(out - ref) / np.abs(ref)
    assert np.max(rel) < 1e-12
