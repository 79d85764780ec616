"""CPU oracle: a plain-numpy restatement of Prometheus's transit integrator.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package (``prometheus_amd``)
imports, calls or links this module.  It is used by ``tests/`` (as the parity
checker), by ``__graft_entry__.smoke()`` (as the checker) and by ``bench.py``'s
``cpu_baseline`` leg (timed, never as the thing measured).

It restates the dataflow of the reference (CrazeXD/Prometheus, mirror at
/root/reference) in functional form.  Every function cites the reference
file:line it follows.  Third-party arithmetic the reference depends on is used
directly (numpy ``interp``/``arange``/``exp``/``add.at``, scipy
``special.voigt_profile`` and ``interpolate.RegularGridInterpolator``); numba is
absent in this image so ``n_interp_log`` is restated with ``np.interp`` (the
survey verified the two bitwise identical on a Na run).

Parity pin: ``tests/test_oracle_golden.py`` checks this module bitwise / to
1e-15 against golden vectors produced by importing the reference itself
(``oracle/gen_golden.py``, fixtures under ``tests/golden/``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

_RES = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "prometheus_amd", "resources")

# --- constants.py:13-26 (cgs, the reference's own values, not CODATA) -------
E_CHARGE = 4.803e-10
M_E = 9.109e-28
C_LIGHT = 2.998e10
G_GRAV = 6.674 * 10 ** (-8)
K_B = 1.381 * 10 ** (-16)
AMU = 1.661 * 10 ** (-24)
R_J = 7.1492e9
M_J = 1.898e30
R_SUN = 6.96e10
M_SUN = 1.988e33
R_IO = 1.822e8
AU = 1.496e13

# constants.py:139-160  name -> (element, ionisation string, mass in amu)
SPECIES = {
    "NaI": ("Na", "1", 22.99), "KI": ("K", "1", 39.0983),
    "SiI": ("Si", "1", 28.0855), "SiII": ("Si", "2", 28.0855),
    "SiIII": ("Si", "3", 28.0855), "SiIV": ("Si", "4", 28.0855),
    "MgI": ("Mg", "1", 24.305), "MgII": ("Mg", "2", 24.305),
    "AlI": ("Al", "1", 26.9815), "CaI": ("Ca", "1", 40.078),
    "CaII": ("Ca", "2", 40.078), "TiI": ("Ti", "1", 47.867),
    "TiII": ("Ti", "2", 47.867), "CrI": ("Cr", "1", 51.9961),
    "MnI": ("Mn", "1", 54.938), "FeI": ("Fe", "1", 55.845),
    "CoI": ("Co", "1", 58.933), "NiI": ("Ni", "1", 58.6934),
    "OI": ("O", "1", 15.999), "CII": ("C", "2", 12.011),
    "SIII": ("S", "3", 32.06), "SIV": ("S", "4", 32.06),
}


def species_mass(name: str) -> float:
    """constants.py:139-160: mass = value * amu (same multiplication order)."""
    return SPECIES[name][2] * AMU


def doppler_shift(v):
    """constants.py:31-45."""
    beta = v / C_LIGHT
    return np.sqrt((1. - beta) / (1. + beta))


# --- line list: gasProperties.py:26-30, :640-670 ------------------------------
_LINE_LIST = None


def line_list() -> np.ndarray:
    global _LINE_LIST
    if _LINE_LIST is None:
        _LINE_LIST = np.loadtxt(os.path.join(_RES, "LineList.txt"), dtype=str,
                                usecols=(0, 1, 2, 3, 4), skiprows=1)
    return _LINE_LIST


def line_parameters(species: str, w_lo: float, w_hi: float):
    """gasProperties.py:640-670 (strict range, A/(4 pi), Angstrom -> cm)."""
    ll = line_list()
    element, ion, _ = SPECIES[species]
    sel = (ll[:, 0] == element) & (ll[:, 1] == ion) & \
        (ll[:, 2] != '') & (ll[:, 3] != '') & (ll[:, 4] != '')
    lam = ll[sel, 2].astype(float) * 1e-8
    gam = ll[sel, 3].astype(float) / (4. * np.pi)
    f = ll[sel, 4].astype(float)
    keep = (lam > min(w_lo, w_hi)) & (lam < max(w_lo, w_hi))
    return lam[keep], gam[keep], f[keep]


# --- wavelength grid: gasProperties.py:990-1071 -------------------------------
def arange_grid(lower, upper, width, res_low, res_high, lines) -> np.ndarray:
    """gasProperties.py:990-1035 (segmented np.arange + sort)."""
    peaks = np.sort(np.unique(lines))
    if len(peaks) == 0:
        return np.arange(lower, upper, res_low)
    gaps = np.concatenate(([np.inf], np.diff(peaks), [np.inf]))
    starts = [p - width / 2. for i, p in enumerate(peaks) if gaps[i] > width]
    stops = [p + width / 2. for i, p in enumerate(peaks) if gaps[i + 1] > width]
    pieces = []
    nwin = len(starts)
    for i in range(nwin):
        pieces.append(np.arange(starts[i], stops[i], res_high))
        if i == 0:
            if lower < starts[0]:
                pieces.append(np.arange(lower, starts[0], res_low))
            if nwin == 1 and upper > stops[-1]:
                pieces.append(np.arange(stops[0], upper, res_low))
        elif i == nwin - 1:
            pieces.append(np.arange(stops[i - 1], starts[i], res_low))
            if upper > stops[-1]:
                pieces.append(np.arange(stops[-1], upper, res_low))
        else:
            pieces.append(np.arange(stops[i - 1], starts[i], res_low))
    return np.sort(np.concatenate(pieces))


def simulation_wavelengths(grid: dict, atomic_species: Sequence[str]) -> np.ndarray:
    """gasProperties.py:1050-1071 (molecules do not shape the grid)."""
    lines: List[float] = []
    for sp in atomic_species:
        lines.extend(line_parameters(sp, grid["lower_w"], grid["upper_w"])[0])
    if len(lines) == 0:
        return np.arange(grid["lower_w"], grid["upper_w"], grid["resolutionLow"])
    return arange_grid(grid["lower_w"], grid["upper_w"], grid["widthHighRes"],
                       grid["resolutionLow"], grid["resolutionHigh"], lines)


# --- cross-section table: gasProperties.py:672-735 ----------------------------
def voigt_sigma(wavelength, species: str, sigma_v: float, w_lo, w_hi):
    """gasProperties.py:672-692 (lines summed in file order, scipy Voigt)."""
    from scipy.special import voigt_profile
    lam0, gam, f = line_parameters(species, w_lo, w_hi)
    sig = np.zeros_like(wavelength)
    for i in range(len(lam0)):
        prof = voigt_profile(C_LIGHT / wavelength - C_LIGHT / lam0[i], sigma_v / lam0[i], gam[i])
        sig += np.pi * E_CHARGE ** 2 / (M_E * C_LIGHT) * f[i] * prof
    return sig


def refined_table(grid: dict, species: str, sigma_v: float, offset=1e-50):
    """gasProperties.py:694-715: resHigh/10, range x(0.99, 1.01), resLow unchanged."""
    lo = grid["lower_w"] * (1. - 0.01)
    hi = grid["upper_w"] * (1. + 0.01)
    lines = line_parameters(species, lo, hi)[0]
    x = arange_grid(lo, hi, grid["widthHighRes"], grid["resolutionLow"],
                    grid["resolutionHigh"] / 10., lines)
    sig = voigt_sigma(x, species, sigma_v, x.min(), x.max())
    return x, np.log10(sig + offset)


def interp_log(targets, xg, yg, offset):
    """gasProperties.py:34-51 (n_interp_log) with numpy interp semantics.

    The reference raises 10 to each *scalar* (``10**log_val`` inside the element
    loop), i.e. libm ``pow``; numpy's vectorised ``np.power`` may dispatch to a
    SIMD pow that differs by an ulp, so the power is taken per element here."""
    v = np.interp(targets, xg, yg)
    p = np.fromiter((10 ** t for t in v.ravel().tolist()), dtype=np.float64, count=v.size)
    return p.reshape(v.shape) - offset


# --- spatial grid: geometryHandler.py:88-208 ----------------------------------
def x_axis(g):
    return np.linspace(g["x_midpoint"] - g["x_border"], g["x_midpoint"] + g["x_border"],
                       int(g["x_steps"]), endpoint=False) + g["x_border"] / float(g["x_steps"])


def rho_axis(g):
    return np.linspace(0., g["upper_rho"], int(g["rho_steps"]), endpoint=False) + \
        0.5 * g["upper_rho"] / float(g["rho_steps"])


def phi_axis(g):
    return np.linspace(0, 2 * np.pi, int(g["phi_steps"]), endpoint=False) + np.pi / float(g["phi_steps"])


def orbphase_axis(g):
    return np.linspace(-g["orbphase_border"], g["orbphase_border"], int(g["orbphase_steps"]))


def delta_x(g):
    return 2. * g["x_border"] / float(g["x_steps"])


def chord_grid(g):
    """geometryHandler.py:188-208 (meshgrid 'ij', orbital phase fastest)."""
    P, R, O = np.meshgrid(phi_axis(g), rho_axis(g), orbphase_axis(g), indexing="ij")
    return np.stack((P.flatten(), R.flatten(), O.flatten()), axis=-1)


# --- bodies: celestialBodies.py -----------------------------------------------
@dataclass
class Body:
    """Planet (+ host star scalars) or moon, as plain numbers."""
    R: float
    M: float
    a: float
    star_R: float = 0.0
    star_M: float = 0.0
    clv_u1: float = 0.0
    clv_u2: float = 0.0
    # host star rotation and spectrum (celestialBodies.py:86-95; Fstar_function's .x / .y)
    vsini: float = 0.0
    phi_rot: float = 0.0
    fstar: Optional[tuple] = None
    # moon only
    host: Optional["Body"] = None
    orbphase0: float = 0.0


def load_planet(name: str) -> Body:
    """celestialBodies.py:597-638 (CSV rows, unit conversions)."""
    import csv
    stars = {}
    with open(os.path.join(_RES, "stars.csv"), newline="") as fh:
        for row in csv.DictReader(fh):
            stars[row["name"]] = (float(row["R_sun"]) * R_SUN, float(row["M_sun"]) * M_SUN)
    with open(os.path.join(_RES, "planets.csv"), newline="") as fh:
        for row in csv.DictReader(fh):
            if row["name"] == name:
                sR, sM = stars[row["hostStar"]]
                return Body(R=float(row["R_J"]) * R_J, M=float(row["M_J"]) * M_J,
                            a=float(row["a_AU"]) * AU, star_R=sR, star_M=sM)
    raise KeyError(name)


def planet_position(p: Body, orb):
    """celestialBodies.py:370-383."""
    return p.a * np.cos(orb), p.a * np.sin(orb)


def planet_los_velocity(p: Body, orb):
    """celestialBodies.py:385-397."""
    return -np.sin(orb) * np.sqrt(G_GRAV * p.star_M / p.a)


def moon_orbphase(m: Body, orb):
    """celestialBodies.py:499-516."""
    a_p = np.float64(m.host.a)
    M_p = np.float64(m.host.M)
    a_m = np.float64(m.a)
    M_s = np.float64(m.host.star_M)
    ratio = np.sqrt((a_p ** 3 * M_p) / (a_m ** 3 * M_s))
    return m.orbphase0 + np.float64(orb) * ratio


def moon_position(m: Body, orb):
    """celestialBodies.py:518-531."""
    om = moon_orbphase(m, orb)
    xp, yp = planet_position(m.host, orb)
    return xp + m.a * np.cos(om), yp + m.a * np.sin(om)


def moon_los_velocity(m: Body, orb):
    """celestialBodies.py:533-550."""
    vp = planet_los_velocity(m.host, orb)
    om = moon_orbphase(m, orb)
    return vp - np.sin(om) * np.sqrt(G_GRAV * m.host.M / m.a)


def _broadcast(x, y, z, bx, by):
    """celestialBodies.py:419-435 batch broadcasting: (n_c,1) against (1,n_x)."""
    return (np.asarray(x)[np.newaxis, :], np.asarray(bx)[:, np.newaxis], np.asarray(by)[:, np.newaxis],
            np.asarray(y)[:, np.newaxis], np.asarray(z)[:, np.newaxis])


def distance_to(bx, by, x, phi, rho):
    """celestialBodies.py:399-436 / :552-583 (batch mode)."""
    y, z = rho * np.sin(phi), rho * np.cos(phi)
    x_, bx_, by_, y_, z_ = _broadcast(x, y, z, bx, by)
    return np.sqrt((x_ - bx_) ** 2 + (y_ - by_) ** 2 + z_ ** 2)


# --- density scenarios: gasProperties.py:53-516 --------------------------------
@dataclass
class Scenario:
    """One density distribution.  kind in
    barometric | hydrostatic | powerLawAtm | powerLawExo | exomoon | torus | serpens | tidal | tabulated."""
    kind: str
    planet: Body
    params: dict
    moon: Optional[Body] = None
    # constituents: list of dicts {"species", "chi", "sigma_v"} (atoms) or
    # {"molecule": table dict, "chi"} (molecules)
    constituents: List[dict] = field(default_factory=list)
    T: float = 0.0
    tabulated_fn: object = None
    grid: object = None   # serpens: (xPoints, yPoints, zPoints, values)

    @property
    def has_moon(self):
        return self.kind in ("exomoon", "tidal")


def number_density(sc: Scenario, x, phi, rho, orb) -> np.ndarray:
    """calculateNumberDensity of every scenario (gasProperties.py:143-516), batch mode."""
    p = sc.planet
    k = sc.kind
    prm = sc.params
    if k == "tabulated":
        return sc.tabulated_fn(x, phi, rho, orb)
    if k == "serpens":                                           # :585-601, one chord at a time
        return np.stack([serpens_density(sc.grid, x, ph, rh) for ph, rh in zip(np.atleast_1d(phi), np.atleast_1d(rho))])
    if k == "tidal":                                             # :440-461
        N = tidal_absorber_number(sc, orb)
        r = distance_to(*moon_position(sc.moon, orb), x, phi, rho)
        N_ = np.asarray(N)
        if N_.ndim > 0:
            N_ = N_[:, np.newaxis]
        n0 = (prm["q"] - 3.) / (4. * np.pi * sc.moon.R ** 3) * N_
        return n0 * (sc.moon.R / r) ** prm["q"] * np.heaviside(r - sc.moon.R, 1.)
    if k in ("barometric", "hydrostatic", "powerLawAtm", "powerLawExo"):
        xp, yp = planet_position(p, orb)
        r = distance_to(xp, yp, x, phi, rho)
        if k == "barometric":                                    # :143-161
            n0 = prm["P_0"] / (K_B * prm["T"])
            H = K_B * prm["T"] * p.R ** 2 / (G_GRAV * prm["mu"] * p.M)
            return n0 * np.exp((p.R - r) / H) * np.heaviside(r - p.R, 1.)
        if k == "hydrostatic":                                   # :185-204
            n0 = prm["P_0"] / (K_B * prm["T"])
            J0 = G_GRAV * prm["mu"] * p.M / (K_B * prm["T"] * p.R)
            J = G_GRAV * prm["mu"] * p.M / (K_B * prm["T"] * r) * np.heaviside(r - p.R, 1.)
            return n0 * np.exp(J - J0)
        if k == "powerLawAtm":                                   # :228-244
            n0 = prm["P_0"] / (K_B * prm["T"])
            return n0 * (p.R / r) ** prm["q"] * np.heaviside(r - p.R, 1.)
        n0 = (prm["q"] - 3.) / (4. * np.pi * p.R ** 3) * prm["N"]  # :311-330
        return n0 * (p.R / r) ** prm["q"] * np.heaviside(r - p.R, 1.)
    if k == "exomoon":                                           # :356-374
        m = sc.moon
        xm, ym = moon_position(m, orb)
        r = distance_to(xm, ym, x, phi, rho)
        n0 = (prm["q"] - 3.) / (4. * np.pi * m.R ** 3) * prm["N"]
        return n0 * (m.R / r) ** prm["q"] * np.heaviside(r - m.R, 1.)
    if k == "torus":                                             # :491-516
        xp, yp = planet_position(p, orb)
        y, z = rho * np.sin(phi), rho * np.cos(phi)
        x_, xp_, yp_, y_, z_ = _broadcast(x, y, z, xp, yp)
        a = np.sqrt((x_ - xp_) ** 2 + (y_ - yp_) ** 2)
        from scipy.special import erf
        at, vej = prm["a_torus"], prm["v_ej"]
        v_orbit = np.sqrt(G_GRAV * p.M / at)
        Ht = at * vej / v_orbit
        n_a = np.exp(-((a - at) / (4. * Ht)) ** 2)
        n_z = np.exp(-(z_ / Ht) ** 2)
        t1 = 8. * Ht ** 2 * np.exp(-at ** 2 / (16. * Ht ** 2))
        t2 = 2. * np.sqrt(np.pi) * at * Ht * (erf(at / (4. * Ht)) + 1.)
        n0 = 1. / (2. * np.pi ** 1.5 * Ht * (t1 + t2)) * prm["N"]
        return n0 * np.multiply(n_a, n_z)
    raise ValueError(k)


# --- SERPENS particle grid: gasProperties.py:548-601 ---------------------------
def serpens_grid(filename, N, g, sigma_smoothing=0.0):
    """addInterpolatedDensity (:548-583): particles [m] -> histogramdd over the x cell edges and
    2 rho_steps sky-plane cells per axis -> density (optionally Gaussian-smoothed) on the cell
    midpoints.  Returns (xPoints, yPoints, zPoints, values)."""
    pos = (np.loadtxt(filename) * 1e2)[:, 0:3]
    lo, hi, n = g["x_midpoint"] - g["x_border"], g["x_midpoint"] + g["x_border"], int(g["x_steps"])
    xb = np.linspace(lo, hi, n + 1)
    rb, nr = g["upper_rho"], int(g["rho_steps"])
    yb = np.linspace(-rb, rb, 2 * nr + 1)
    zb = np.linspace(-rb, rb, 2 * nr + 1)
    vol = (xb[1] - xb[0]) * (yb[1] - yb[0]) * (zb[1] - zb[0])
    vals = np.histogramdd(pos, bins=[xb, yb, zb])[0] * N / (np.size(pos, axis=0) * vol)
    if sigma_smoothing > 0.:
        from scipy.ndimage import gaussian_filter
        vals = gaussian_filter(vals, sigma=sigma_smoothing)
    xp = np.linspace(lo, hi, n, endpoint=False) + g["x_border"] / float(n)
    yp = np.linspace(-rb, rb, 2 * nr, endpoint=False) + 2. * rb / (4. * nr)
    zp = np.linspace(-rb, rb, 2 * nr, endpoint=False) + 2. * rb / (4. * nr)
    return xp, yp, zp, vals


def serpens_density(grid, x, phi, rho):
    """calculateNumberDensity (:585-601) for one chord: scipy RegularGridInterpolator (linear,
    bounds_error=True) at (x, rho sin phi, rho cos phi)."""
    from scipy.interpolate import RegularGridInterpolator
    xp, yp, zp, vals = grid
    y, z = rho * np.sin(phi), rho * np.cos(phi)
    pts = np.array([x, np.repeat(y, np.size(x)), np.repeat(z, np.size(x))]).T
    return RegularGridInterpolator((xp, yp, zp), vals)(pts)


# --- tidally heated moon: gasProperties.py:377-461 -----------------------------
def tidal_source(filename, tau_photoionization, mass_absorber):
    """addSourceRateFunction (:404-424): the mirrored M_dot profile on [0, 2 pi] -> log10 N nodes."""
    mdot = np.loadtxt(filename)
    mdot = np.concatenate((mdot, mdot[::-1]))
    return np.linspace(0., 2. * np.pi, len(mdot)), np.log10(mdot * tau_photoionization / mass_absorber)


def tidal_absorber_number(sc, orb):
    """calculateAbsorberNumber (:426-438): 10^interp1d(phi_moon, log10 N) at the moon's phase mod 2 pi
    (scipy interp1d, linear: bracket from searchsorted-left clipped to [1, n-1])."""
    from scipy.interpolate import interp1d
    xs, ys = sc.params["source"]
    om = moon_orbphase(sc.moon, orb) % (2. * np.pi)
    return 10 ** interp1d(xs, ys)(om)


# --- molecular table: gasProperties.py:765-818 ---------------------------------
def molecular_interpolator(table: dict, offset=1e-50):
    """gasProperties.py:774-781 (P*10, lambda = 1/nu reversed, log10 table)."""
    from scipy.interpolate import RegularGridInterpolator
    P = np.asarray(table["p"]) * 10.
    T = np.asarray(table["t"])
    lam = 1. / np.asarray(table["bin_edges"])[::-1]
    sig = np.asarray(table["xsecarr"])[:, :, ::-1]
    return RegularGridInterpolator((P, T, lam), np.log10(sig + offset), bounds_error=False,
                                   fill_value=np.log10(offset))


def molecular_sigma(rgi, P, T, wav, offset=1e-50):
    """gasProperties.py:789-818: (n_c, n_x, n_wav) sigma, P clipped at 1e-4."""
    nc, nw = wav.shape
    nx = P.shape[1]
    tot = nc * nx * nw
    Pf = np.clip(np.broadcast_to(P[:, :, None], (nc, nx, nw)).reshape(tot), 1e-4, None)
    wf = np.broadcast_to(wav[:, None, :], (nc, nx, nw)).reshape(tot)
    pts = np.column_stack([Pf, np.full(tot, T), wf])
    return (10 ** rgi(pts) - offset).reshape(nc, nx, nw)


# --- C restatement of the molecular optical depth (oracle/mol_tau.c) -------------
_MOL_C = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmol_tau.so")


def build_c(force=False):
    """gcc -O2 -fopenmp oracle/mol_tau.c -> oracle/libmol_tau.so (test infrastructure; no -ffast-math:
    the restatement keeps IEEE order)."""
    import subprocess
    src = os.path.join(os.path.dirname(_MOL_C), "mol_tau.c")
    if force or not os.path.exists(_MOL_C) or os.path.getmtime(_MOL_C) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-fno-fast-math", "-ffp-contract=off", "-fopenmp", "-shared",
                               "-fPIC", src, "-o", _MOL_C, "-lm"])
    return _MOL_C


def molecular_tau_c(rgi, n_chi, P, T, shifts, wav, dx, tau, offset=1e-50):
    """tau += dx * einsum("cx,cxw->cw", n_chi, molecular_sigma(rgi, P, T, shifts[:, None] * wav[None, :]))
    through oracle/mol_tau.c (same interpolation semantics and order; OpenMP over chords)."""
    import ctypes
    lib = ctypes.CDLL(build_c())
    f = lib.oracle_mol_tau
    dp = ctypes.POINTER(ctypes.c_double)
    i64, dbl = ctypes.c_int64, ctypes.c_double
    f.argtypes = [i64, i64, i64, dp, dp, dp, dp, i64, dp, i64, dp, i64, dp, dp, dbl, dbl, dbl, dbl, dp]
    f.restype = None
    Pg, Tg, lg = (np.ascontiguousarray(g, dtype=np.float64) for g in rgi.grid)
    vals = np.ascontiguousarray(rgi.values, dtype=np.float64)
    n1 = np.ascontiguousarray(n_chi, dtype=np.float64)
    P1 = np.ascontiguousarray(np.broadcast_to(P, n1.shape), dtype=np.float64)
    sh = np.ascontiguousarray(shifts, dtype=np.float64)
    w1 = np.ascontiguousarray(wav, dtype=np.float64)
    assert tau.flags.c_contiguous and tau.dtype == np.float64 and tau.shape == (n1.shape[0], len(w1))
    ptr = lambda a: a.ctypes.data_as(dp)  # noqa: E731
    f(n1.shape[0], n1.shape[1], len(w1), ptr(n1), ptr(P1), ptr(sh), ptr(w1), len(Pg), ptr(Pg), len(Tg), ptr(Tg),
      len(lg), ptr(lg), ptr(vals), float(T), float(offset), 1.0, float(dx), ptr(tau))


# --- optical depth: gasProperties.py:885-956 -----------------------------------
def optical_depth(scenarios, doppler, x, phi, rho, orb, wav, dx, tables, mol_c=False):
    """Atmosphere.getLOSopticalDepth_Batch restated.  ``tables[(si, ci)]`` holds
    (x, y) refined log-sigma tables for atoms or an RGI for molecules (``mol_c``: molecular constituents
    through oracle/mol_tau.c, the same interpolation restated in C)."""
    nc = len(phi)
    tau = np.zeros((nc, len(wav)))
    for si, sc in enumerate(scenarios):
        if doppler:
            v = moon_los_velocity(sc.moon, orb) if sc.has_moon else planet_los_velocity(sc.planet, orb)
        else:
            v = np.zeros(nc)
        shifts = doppler_shift(-v)
        n_tot = number_density(sc, x, phi, rho, orb)
        for ci, con in enumerate(sc.constituents):
            if "molecule" in con:
                P = n_tot * K_B * sc.T
                if mol_c:
                    molecular_tau_c(tables[(si, ci)], n_tot * con["chi"], P, sc.T, shifts, wav, dx, tau)
                    continue
                sig = molecular_sigma(tables[(si, ci)], P, sc.T, shifts[:, None] * wav[None, :])
                tau += np.einsum("cx,cxw->cw", n_tot * con["chi"], sig) * dx
            else:
                col = np.sum(n_tot * con["chi"], axis=1) * dx
                us, inv = np.unique(shifts, return_inverse=True)
                xg, yg = tables[(si, ci)]
                sig = interp_log(us[:, None] * wav[None, :], xg, yg, 1e-50)[inv]
                tau += col[:, None] * sig
    return tau


def chunk_size(n_chords, n_wav, n_x, max_memory_gb, molecular):
    """memoryHandler.py:13-66 (psutil-free: the limit is max_memory_gb)."""
    per = (n_x * n_wav * 64 if molecular else n_wav * 16) * 2.0
    return min(max(1, int(int(max_memory_gb * 1e9) / int(per))), n_chords)


def transit_depth(scenarios, doppler, grid, wav, tables, max_memory_gb=2.0,
                  chord_limit=None, mol_c=False):
    """Transit.sumOverChords restated (gasProperties.py:1160-1258).

    ``chord_limit`` (bench CPU-baseline sample only) truncates the chord list
    after that many chords; R is then a partial-disk ratio."""
    cg = chord_grid(grid)
    if chord_limit is not None:
        cg = cg[:chord_limit]
    planet = scenarios[0].planet
    n_wav = len(wav)
    n_orb = int(grid["orbphase_steps"])
    phi, rho, orb = cg[:, 0], cg[:, 1], cg[:, 2]
    y, z = rho * np.sin(phi), rho * np.cos(phi)
    orb_idx = np.abs(orb[:, None] - orbphase_axis(grid)).argmin(axis=1)
    mu = np.sqrt(np.clip(1. - rho ** 2 / planet.star_R ** 2, 0, 1))
    clv = 1. - planet.clv_u1 * (1. - mu) - planet.clv_u2 * (1. - mu) ** 2
    # gasProperties.py:1183-1184
    star_shifts = doppler_shift(planet.vsini * rho / planet.star_R * np.cos(phi - planet.phi_rot))
    molecular = any("molecule" in c for s in scenarios for c in s.constituents)
    x = x_axis(grid)
    B = chunk_size(len(cg), n_wav, len(x), max_memory_gb, molecular and not mol_c)
    dx = delta_x(grid)
    Fin = np.zeros((n_orb, n_wav))
    Fout = np.zeros((n_orb, n_wav))
    for i in range(0, len(cg), B):
        s = slice(i, i + B)
        if planet.fstar is None:                       # gasProperties.py:1210-1211
            Fstar = np.ones((len(phi[s]), n_wav))
        else:                                          # :1212-1219
            Fstar = interp_log(wav[None, :] / star_shifts[s, None], planet.fstar[0], planet.fstar[1], 0.0)
        Fstar *= clv[s, None]
        blocked = np.sqrt((y[s] - planet.a * np.sin(orb[s])) ** 2 + z[s] ** 2) < planet.R
        for sc in scenarios:
            if sc.has_moon:
                ym = moon_position(sc.moon, orb[s])[1]
                blocked |= ((y[s] - ym) ** 2 + z[s] ** 2 < sc.moon.R ** 2)
        fo = rho[s, None] * Fstar
        fi = np.zeros_like(fo)
        act = ~blocked
        if np.any(act):
            tau = optical_depth(scenarios, doppler, x, phi[s][act], rho[s][act], orb[s][act],
                                wav, dx, tables, mol_c)
            fi[act] = fo[act] * np.exp(-tau)
        if B == len(cg) and chord_limit is None:
            npr = int(grid["phi_steps"]) * int(grid["rho_steps"])
            Fin = fi.reshape(npr, n_orb, n_wav).sum(axis=0)
            Fout = fo.reshape(npr, n_orb, n_wav).sum(axis=0)
        else:
            np.add.at(Fin, orb_idx[s], fi)
            np.add.at(Fout, orb_idx[s], fo)
    return Fin / Fout


def lightcurve(R, wav, orbphase, planet: Body, centers=(5891.583253e-8, 5897.558147e-8), bandwidth=0.75e-8):
    """Band-averaged light curve restated from mainRetrieval.py:76-93: per phase, mean of R over the
    wavelengths within +-bandwidth/2 (inclusive) of any line centre times the planet's Doppler factor,
    divided by the maximum of R at that phase."""
    shift = doppler_shift(planet_los_velocity(planet, np.asarray(orbphase)))
    out = []
    for i in range(len(orbphase)):
        sel = np.zeros(len(wav), dtype=bool)
        for c in centers:
            sel |= (wav >= c * shift[i] - bandwidth / 2.) & (wav <= c * shift[i] + bandwidth / 2.)
        out.append(np.mean(R[i, sel]) / np.max(R[i, :]))
    return np.array(out)


def build_tables(scenarios, grid):
    """Per-constituent lookup tables (gasProperties.py:717-725, :783-787)."""
    tabs = {}
    for si, sc in enumerate(scenarios):
        for ci, con in enumerate(sc.constituents):
            if "molecule" in con:
                tabs[(si, ci)] = molecular_interpolator(con["molecule"])
            else:
                tabs[(si, ci)] = refined_table(grid, con["species"], con["sigma_v"])
    return tabs


def atomic_species(scenarios):
    return [c["species"] for s in scenarios for c in s.constituents if "molecule" not in c]


def thermal_sigma_v(T, species):
    """gasProperties.py:86-96."""
    return np.sqrt(T * K_B / species_mass(species))


def synthetic_molecular_table(n_p=22, n_t=27, n_nu=50001, nu_lo=5000., nu_hi=10000., seed=0):
    """Seeded ExoMol/TauREx-layout table (p [Pa], t [K], bin_edges [cm^-1], xsecarr[p,t,nu])."""
    rng = np.random.default_rng(seed)
    return {"p": np.logspace(-1, 8, n_p), "t": np.linspace(100., 3400., n_t),
            "bin_edges": np.linspace(nu_lo, nu_hi, n_nu),
            "xsecarr": 1e-22 * np.exp(rng.standard_normal((n_p, n_t, n_nu)))}


# --- setup-file loader: prometheus.py:59-134 ------------------------------------
def from_setup(cfg: dict, molecular_tables: Optional[dict] = None):
    """Scenario objects from a setup dict, restating prometheus.py:66-131.

    Returns (scenarios, doppler, grids).  ``molecular_tables`` maps a molecule
    name to a TauREx-layout dict (stands in for ../molecularResources/<mol>.h5)."""
    arch, scen, spec, grids = cfg["Architecture"], cfg["Scenarios"], cfg["Species"], cfg["Grids"]
    planet = load_planet(arch["planetName"])
    out = []
    for key, prm in scen.items():
        if key == "barometric":
            sc = Scenario("barometric", planet, {"T": prm["T"], "P_0": prm["P_0"], "mu": prm["mu"]})
        elif key == "hydrostatic":
            sc = Scenario("hydrostatic", planet, {"T": prm["T"], "P_0": prm["P_0"], "mu": prm["mu"]})
        elif key == "powerLaw":
            if "P_0" in prm:
                sc = Scenario("powerLawAtm", planet, {"T": prm["T"], "P_0": prm["P_0"], "q": prm["q_esc"]})
            else:
                first = list(spec["powerLaw"].keys())[0]
                sc = Scenario("powerLawExo", planet, {"N": spec["powerLaw"][first]["Nparticles"],
                                                      "q": prm["q_esc"]})
        elif key == "exomoon":
            moon = Body(R=arch["R_moon"], M=0.0, a=arch["a_moon"], host=planet,
                        orbphase0=arch["starting_orbphase_moon"])
            first = list(spec["exomoon"].keys())[0]
            sc = Scenario("exomoon", planet, {"N": spec["exomoon"][first]["Nparticles"],
                                              "q": prm["q_moon"]}, moon=moon)
        elif key == "torus":
            first = list(spec["torus"].keys())[0]
            sc = Scenario("torus", planet, {"N": spec["torus"][first]["Nparticles"],
                                            "a_torus": prm["a_torus"], "v_ej": prm["v_ej"]})
        elif key == "serpens":
            first = list(spec["serpens"].keys())[0]
            N = spec["serpens"][first]["Nparticles"]
            sc = Scenario("serpens", planet, {"N": N})
            sc.grid = serpens_grid(prm["serpensPath"], N, grids, 0.)   # sigmaSmoothing 0 (prometheus.py:103)
        else:
            raise ValueError("scenario %r is not restated by the oracle" % key)
        collisional = "T" in prm
        for name, ab in spec[key].items():
            if name in SPECIES:
                if collisional:
                    sc.constituents.append({"species": name, "chi": ab["chi"],
                                            "sigma_v": thermal_sigma_v(prm["T"], name)})
                else:
                    sc.constituents = [{"species": name, "chi": 1., "sigma_v": ab["sigma_v"]}]
            else:
                tab = (molecular_tables or {})[name]
                if collisional:
                    sc.constituents.append({"molecule": tab, "chi": ab["chi"]})
                    sc.T = prm["T"]
                else:
                    sc.constituents = [{"molecule": tab, "chi": 1.0}]
                    sc.T = ab["T"]
        if collisional:
            sc.T = prm["T"]
        out.append(sc)
    return out, bool(cfg["Fundamentals"]["DopplerOrbitalMotion"]), grids


def apply_star(planet: Body, star: Optional[dict]) -> None:
    """Star.addCLVparameters / addRMparameters / Fstar_function (celestialBodies.py:76-95, :223-235):
    ``star`` = {"u1", "u2", "vsini", "phi_rot", "fstar": (x, log10 F) or None}."""
    if not star:
        return
    planet.clv_u1, planet.clv_u2 = star.get("u1", 0.0), star.get("u2", 0.0)
    planet.vsini, planet.phi_rot = star.get("vsini", 0.0), star.get("phi_rot", 0.0)
    planet.fstar = star.get("fstar")


def star_disk_flux(x, logF, R_star, u1, u2, vsini, phi_rot, phi_axis, rho_axis, dphi, drho, wavelength):
    """Star.getFstarIntegrated, rotating branch (celestialBodies.py:299-311): cells in the reference's loop
    order (phi outer, rho inner), F = 10**interp1d(x, logF)(lambda / shift) (calculateRM :226-240, interp1d
    linear = numpy.interp in range), times calculateCLV (:212-224), accumulated one cell after the other."""
    wavelength = np.asarray(wavelength, dtype=np.float64)
    acc = np.zeros_like(wavelength)
    for phi in phi_axis:
        for rho in rho_axis:
            v = vsini * rho / R_star * np.cos(phi - phi_rot)
            shift = doppler_shift(v)
            t = wavelength / shift
            if np.any(t < x[0]) or np.any(t > x[-1]):
                raise ValueError("target outside the stellar spectrum (interp1d bounds_error)")
            F = 10. ** np.interp(t, x, logF)
            arg = 1. - np.sqrt(1. - rho ** 2 / R_star ** 2)
            F *= 1. - u1 * arg - u2 * arg ** 2
            acc += F * dphi * drho * rho
    return acc


def synthetic_star_spectrum(lower_w, upper_w, step=1e-10, margin=3e-8, seed=7):
    """Seeded stand-in for a PHOENIX HiRes slice (the reference fetches it over FTP,
    celestialBodies.py:128-209; no network here): x = arange(lower_w - margin, upper_w + margin, step)
    [cm], F = continuum with a 10 % slope times one Gaussian absorption line per 2 A (depth 5-90 %,
    sigma 0.05-0.4 A) -> (x, F).  Same formula as prometheus_amd.configs.synthetic_star_spectrum."""
    rng = np.random.default_rng(seed)
    x = np.arange(lower_w - margin, upper_w + margin, step)
    n_lines = max(4, int((x[-1] - x[0]) / 2e-8))
    centre = rng.uniform(x[0], x[-1], n_lines)
    depth = rng.uniform(0.05, 0.9, n_lines)
    width = rng.uniform(0.05e-8, 0.4e-8, n_lines)
    F = 2e14 * (1. + 0.1 * (x - x[0]) / (x[-1] - x[0]))
    for c, d, w in zip(centre, depth, width):
        a, b = np.searchsorted(x, [c - 8. * w, c + 8. * w])
        F[a:b] *= 1. - d * np.exp(-0.5 * ((x[a:b] - c) / w) ** 2)
    return x, F


def run_setup(cfg: dict, molecular_tables: Optional[dict] = None, max_memory_gb=2.0, star=None):
    """prometheus.py:131-143 equivalent: returns (wavelength, orbphase, R).  ``star``: apply_star."""
    scen, doppler, grids = from_setup(cfg, molecular_tables)
    apply_star(scen[0].planet, star)
    tabs = build_tables(scen, grids)
    wav = simulation_wavelengths(grids, atomic_species(scen))
    R = transit_depth(scen, doppler, grids, wav, tabs, max_memory_gb)
    return wav, orbphase_axis(grids), R
