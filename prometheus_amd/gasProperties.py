"""Gas properties and the transit integrator (mirrors ``pythonScripts/gasProperties.py``).

Same classes, method names and argument meanings as the reference, so scripts written for
``pythonScripts.gasProperties`` run unchanged against ``prometheus_amd.gasProperties``.  What
changes is where the arithmetic runs:

* density plugins, Voigt cross-section tables, sigma lookups and the whole
  ``Transit.sumOverChords`` integral run as HIP kernels on MI355X through the C-ABI of
  ``libprom_hip.so`` (``_native.py``); there is no CPU fallback -- without the library or a
  GPU these calls raise ``NativeUnavailable``;
* host code does what the reference's host code does and nothing heavier: it parses the line
  list, builds the wavelength nodes with the same numpy ``arange``/``sort`` calls (so every node
  is bit-identical), and evaluates O(n_orbphase) / O(n_chord-positions) scalars (orbital
  positions, Doppler factors, limb darkening) with numpy.

Wavelength sharding: ``sumOverChords(devices=[...])`` splits the wavelength axis into
contiguous shards, one host thread per GPU, and gathers R on the host (no collective).
Per-wavelength arithmetic does not depend on the split, so R is bitwise identical for any
number of devices.
"""
from __future__ import annotations

import math
import os
import threading
import weakref
from copy import deepcopy
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _native
from . import constants as const
from . import geometryHandler as geom
from .sharding import WAVE_ALIGN, split as _split   # shard / chunk edges

_HERE = os.path.dirname(os.path.abspath(__file__))
lineListPath: str = os.path.join(_HERE, "resources", "LineList.txt")
LINE_LIST = np.loadtxt(lineListPath, dtype=str, usecols=(0, 1, 2, 3, 4), skiprows=1)
# the reference looks for <parent of the checkout>/molecularResources/<name>.h5 (gasProperties.py:31-32)
molecularLookupPath: str = os.environ.get(
    "PROMETHEUS_MOLECULAR_PATH", os.path.join(os.path.dirname(os.path.dirname(_HERE)), "molecularResources"))

_MOLECULAR_TABLES: Dict[str, dict] = {}


def register_molecular_table(name: str, table: dict) -> None:
    """Provide an ExoMol/TauREx-layout table in memory: keys p [Pa], t [K], bin_edges [cm^-1],
    xsecarr[p][t][nu] [cm^2].  Takes precedence over files in ``molecularLookupPath``."""
    _MOLECULAR_TABLES[name] = table


def _device(dev=None):
    return _native.get_device(_native.default_device() if dev is None else dev)


def _release_tables(ids: Dict[int, int], molecular: bool) -> None:
    """Finalizer of a table object: its device copies are freed at the context's next upload."""
    for d, tid in list(ids.items()):
        dev = _native._contexts.get(d)   # never create a context from a finalizer
        if dev is not None:
            dev.release_later(molecular, tid)
    ids.clear()


class LookupTable:
    """Host copy of a log10-sigma table (the reference keeps an interp1d with .x/.y) plus its
    device-resident copies, one per GPU, uploaded on first use and freed when the object is
    collected."""

    def __init__(self, x: np.ndarray, y: np.ndarray, offset: float, ids: Optional[Dict[int, int]] = None):
        self.x = x
        self.y = y
        self.offset = offset
        self._ids: Dict[int, int] = dict(ids or {})
        self._lock = threading.Lock()
        weakref.finalize(self, _release_tables, self._ids, False)

    def __deepcopy__(self, memo):
        # a copy owns no device ids (it uploads its own on first use); sharing them would leave it
        # reading a table freed when this object is collected
        return LookupTable(deepcopy(self.x, memo), deepcopy(self.y, memo), self.offset)

    def table_id(self, dev: "_native.Device") -> int:
        with self._lock:
            tid = self._ids.get(dev.device)
            if tid is None:
                tid = dev.table_upload(self.x, self.y, self.offset)
                self._ids[dev.device] = tid
            return tid


def n_interp_log(x_targets, x_grid, y_grid_log, offset):
    """10^interp(x_targets; x_grid, y_grid_log) - offset on the GPU (gasProperties.py:34-51)."""
    dev = _device()
    with dev.lock:
        tid = dev.table_upload(x_grid, y_grid_log, offset)
        try:
            t = np.asarray(x_targets, dtype=np.float64)
            return dev.table_lookup(tid, t.ravel()).reshape(t.shape)
        finally:
            dev.table_free(tid)


# ============================================================================== density scenarios
class CollisionalAtmosphere:
    """Isothermal atmosphere with temperature T [K] and reference pressure P_0 [dyn cm^-2]."""

    def __init__(self, T: float, P_0: float):
        self.T = T
        self.P_0 = P_0
        self.constituents: List[Any] = []
        self.hasMoon = False

    def getReferenceNumberDensity(self) -> float:
        return self.P_0 / (const.k_B * self.T)

    def getVelDispersion(self, m: float) -> float:
        return np.sqrt(self.T * const.k_B / m)

    def addConstituent(self, speciesName: str, chi: float) -> None:
        species = const.AvailableSpecies().findSpecies(speciesName)
        self.constituents.append(AtmosphericConstituent(species, chi, self.getVelDispersion(species.mass)))

    def addMolecularConstituent(self, speciesName: str, chi: float) -> None:
        self.constituents.append(MolecularConstituent(speciesName, chi))

    # --- device side ---
    def densityModel(self) -> Tuple[int, List[float], Any]:
        """(prom_density_kind, scalar parameters, body whose getPosition centres the profile)."""
        raise NotImplementedError

    def calculateNumberDensity(self, x, phi, rho, orbphase):
        return _device_density(self, x, phi, rho, orbphase)


def _device_density(model, x, phi, rho, orbphase):
    """calculateNumberDensity of a built-in scenario, evaluated by prom_number_density."""
    kind, params, body = model.densityModel()
    x = np.asarray(x, dtype=np.float64)
    scalar = np.ndim(phi) == 0 and np.ndim(rho) == 0 and np.ndim(orbphase) == 0
    phi_, rho_, orb_ = np.broadcast_arrays(np.atleast_1d(phi), np.atleast_1d(rho), np.atleast_1d(orbphase))
    y, z = geom.Grid.getCartesianFromCylinder(phi_, rho_)
    bx, by = body.getPosition(orb_)
    dev = _device()
    with dev.lock:
        n = dev.number_density(kind, params, x, y, z, np.broadcast_to(bx, y.shape), np.broadcast_to(by, y.shape))
    return n[0] if scalar else n


class BarometricAtmosphere(CollisionalAtmosphere):
    """n = n_0 exp((R - r)/H) Heaviside(r - R),  H = k_B T R^2 / (G mu M)  (gasProperties.py:122-161)."""

    def __init__(self, T: float, P_0: float, mu: float, planet: Any):
        super().__init__(T, P_0)
        self.mu = mu
        self.planet = planet

    def densityModel(self):
        n0 = self.getReferenceNumberDensity()
        H = const.k_B * self.T * self.planet.R ** 2 / (const.G * self.mu * self.planet.M)
        return _native.DENSITY_BAROMETRIC, [n0, self.planet.R, H], self.planet


class HydrostaticAtmosphere(CollisionalAtmosphere):
    """n = n_0 exp(J(r) Heaviside(r - R) - J_0),  J = G mu M / (k_B T r)  (gasProperties.py:164-204)."""

    def __init__(self, T: float, P_0: float, mu: float, planet: Any):
        super().__init__(T, P_0)
        self.mu = mu
        self.planet = planet

    def densityModel(self):
        n0 = self.getReferenceNumberDensity()
        gmm = const.G * self.mu * self.planet.M
        kt = const.k_B * self.T
        j0 = const.G * self.mu * self.planet.M / (const.k_B * self.T * self.planet.R)
        return _native.DENSITY_HYDROSTATIC, [n0, self.planet.R, gmm, kt, j0], self.planet


class PowerLawAtmosphere(CollisionalAtmosphere):
    """n = n_0 (R/r)^q Heaviside(r - R), pressure-normalised  (gasProperties.py:207-244)."""

    def __init__(self, T: float, P_0: float, q: float, planet: Any):
        super().__init__(T, P_0)
        self.q = q
        self.planet = planet

    def densityModel(self):
        return _native.DENSITY_POWERLAW, [self.getReferenceNumberDensity(), self.planet.R, self.q], self.planet


class EvaporativeExosphere:
    """Exosphere normalised by its total particle number N; one absorber (gasProperties.py:247-288)."""

    def __init__(self, N: float):
        self.N = N
        self.hasMoon = False

    def addConstituent(self, speciesName: str, sigma_v: float) -> None:
        species = const.AvailableSpecies().findSpecies(speciesName)
        self.constituents = [AtmosphericConstituent(species, 1., sigma_v)]

    def addMolecularConstituent(self, speciesName: str, T: float) -> None:
        self.constituents = [MolecularConstituent(speciesName, 1.0)]
        self.T = T

    def densityModel(self):
        raise NotImplementedError

    def calculateNumberDensity(self, x, phi, rho, orbphase):
        return _device_density(self, x, phi, rho, orbphase)


class PowerLawExosphere(EvaporativeExosphere):
    """n = (q-3)/(4 pi R^3) N (R/r)^q Heaviside(r - R)  (gasProperties.py:291-330)."""

    def __init__(self, N: float, q: float, planet: Any):
        super().__init__(N)
        self.q = q
        self.planet = planet

    def densityModel(self):
        n0 = (self.q - 3.) / (4. * np.pi * self.planet.R ** 3) * self.N
        return _native.DENSITY_POWERLAW, [n0, self.planet.R, self.q], self.planet


class MoonExosphere(EvaporativeExosphere):
    """Power law about an exomoon; the moon also blocks light (gasProperties.py:333-374)."""

    def __init__(self, N: float, q: float, moon: Any):
        super().__init__(N)
        self.q = q
        self.moon = moon
        self.hasMoon = True
        self.planet = moon.hostPlanet

    def densityModel(self):
        n0 = (self.q - 3.) / (4. * np.pi * self.moon.R ** 3) * self.N
        return _native.DENSITY_POWERLAW, [n0, self.moon.R, self.q], self.moon


class TidallyHeatedMoon(EvaporativeExosphere):
    """Moon exosphere with a phase-dependent source rate (gasProperties.py:377-461).

    Not a built-in device scenario: its density is evaluated on the host by the plugin itself
    (``calculateNumberDensity``, numpy/scipy as in the reference) and handed to the device as a
    tabulated n(c, x) (PROM_DENSITY_TABULATED), like any user plugin."""

    def __init__(self, q: float, moon: Any):
        self.q = q
        self.moon = moon
        self.hasMoon = True
        self.planet = moon.hostPlanet

    def addSourceRateFunction(self, filename: str, tau_photoionization: float, mass_absorber: float) -> None:
        """M_dot(moon phase) from a file, mirrored onto [0, 2 pi]; N = M_dot tau / m (:404-424)."""
        from scipy.interpolate import interp1d
        mdot = np.loadtxt(filename)
        mdot = np.concatenate((mdot, mdot[::-1]))
        phi_moon = np.linspace(0., 2. * np.pi, len(mdot))
        self.N_function = interp1d(phi_moon, np.log10(mdot * tau_photoionization / mass_absorber))

    def calculateAbsorberNumber(self, orbphase):
        """N = 10^N_function(moon phase mod 2 pi) (:426-438; scipy interp1d, as the reference)."""
        om = self.moon.getOrbphase(orbphase) % (2. * np.pi)
        return 10 ** self.N_function(om)

    def calculateNumberDensity(self, x, phi, rho, orbphase):
        N = np.asarray(self.calculateAbsorberNumber(orbphase))
        r = self.moon.getDistanceFromMoon(x, phi, rho, orbphase)
        if N.ndim > 0:
            N = N[:, np.newaxis]
        n0 = (self.q - 3.) / (4. * np.pi * self.moon.R ** 3) * N
        return n0 * (self.moon.R / r) ** self.q * np.heaviside(r - self.moon.R, 1.)


class TorusExosphere(EvaporativeExosphere):
    """Gaussian torus of radius a_torus and scale height a v_ej / v_orbit (gasProperties.py:464-516)."""

    def __init__(self, N: float, a_torus: float, v_ej: float, planet: Any):
        super().__init__(N)
        self.a_torus = a_torus
        self.v_ej = v_ej
        self.planet = planet

    def densityModel(self):
        v_orbit = np.sqrt(const.G * self.planet.M / self.a_torus)
        H = self.a_torus * self.v_ej / v_orbit
        t1 = 8. * H ** 2 * np.exp(-self.a_torus ** 2 / (16. * H ** 2))
        t2 = 2. * np.sqrt(np.pi) * self.a_torus * H * (math.erf(self.a_torus / (4. * H)) + 1.)
        n0 = 1. / (2. * np.pi ** 1.5 * H * (t1 + t2)) * self.N
        return _native.DENSITY_TORUS, [n0, self.a_torus, 4. * H, H], self.planet


class SerpensExosphere(EvaporativeExosphere):
    """SERPENS particle cloud (gasProperties.py:519-601): the particles are histogrammed onto a 3-D grid
    (numpy, once, as the reference does) and the density is scipy's RegularGridInterpolator (linear) of
    that grid, sampled on the device (PROM_DENSITY_GRIDDED, ``prom_gridded_density``).

    The grid is fixed in the star frame: the density does not depend on the orbital phase
    (``calculateNumberDensity`` ignores ``orbphase``, :587-601).  Unlike the reference, whose
    ``calculateNumberDensity`` builds a ragged coordinate array for batched chords and fails inside
    ``getLOSopticalDepth_Batch`` (:905), chords may be batched: phi, rho of shape (B,) give n of shape
    (B, n_x), each row equal to the reference's scalar call for that chord."""

    def __init__(self, filename: str, N: float, planet: Any, sigmaSmoothing: float):
        super().__init__(N)
        self.filename = filename
        self.planet = planet
        self.sigmaSmoothing = sigmaSmoothing

    def addInterpolatedDensity(self, spatialGrid: Any) -> None:
        """Histogram the SERPENS particles (file in m, one particle per row, x y z first) onto the
        spatial grid's cells and keep the grid for the device sampler (:548-583)."""
        serpensOutput = np.loadtxt(self.filename) * 1e2
        particlePos = serpensOutput[:, 0:3]
        xBins = spatialGrid.constructXaxis(midpoints=False)
        yBins = np.linspace(-spatialGrid.rho_border, spatialGrid.rho_border, 2 * int(spatialGrid.rho_steps) + 1)
        zBins = np.linspace(-spatialGrid.rho_border, spatialGrid.rho_border, 2 * int(spatialGrid.rho_steps) + 1)
        cellVolume = (xBins[1] - xBins[0]) * (yBins[1] - yBins[0]) * (zBins[1] - zBins[0])
        n_histogram = np.histogramdd(particlePos, bins=[xBins, yBins, zBins])[0] * self.N / (
            np.size(particlePos, axis=0) * cellVolume)
        if self.sigmaSmoothing > 0.:
            from scipy.ndimage import gaussian_filter
            n_histogram = gaussian_filter(n_histogram, sigma=self.sigmaSmoothing)
        xPoints = spatialGrid.constructXaxis()
        half = 2. * spatialGrid.rho_border / (4. * spatialGrid.rho_steps)
        yPoints = np.linspace(-spatialGrid.rho_border, spatialGrid.rho_border, 2 * int(spatialGrid.rho_steps),
                              endpoint=False) + half
        zPoints = np.linspace(-spatialGrid.rho_border, spatialGrid.rho_border, 2 * int(spatialGrid.rho_steps),
                              endpoint=False) + half
        self.gridAxes = tuple(np.ascontiguousarray(a, dtype=np.float64) for a in (xPoints, yPoints, zPoints))
        self.gridValues = np.ascontiguousarray(n_histogram, dtype=np.float64)
        self._packed = np.concatenate(self.gridAxes + (self.gridValues.ravel(),))

    def _require_grid(self):
        if not hasattr(self, "gridValues"):
            raise AttributeError("SerpensExosphere: call addInterpolatedDensity(spatialGrid) first "
                                 "(prometheus.py:103-104)")

    def checkBounds(self, x, y, z) -> None:
        """RegularGridInterpolator's bounds_error (scipy _rgi.py _prepare_xi): every coordinate inside
        [axis[0], axis[-1]], else ValueError naming the first offending dimension."""
        self._require_grid()
        for i, (ax, p) in enumerate(zip(self.gridAxes, (x, y, z))):
            p = np.asarray(p, dtype=np.float64)
            if not np.logical_and(np.all(ax[0] <= p), np.all(p <= ax[-1])):
                raise ValueError("One of the requested xi is out of bounds in dimension %d" % i)

    def densityModel(self):
        self._require_grid()
        nx, ny, nz = (len(a) for a in self.gridAxes)
        return _native.DENSITY_GRIDDED, [nx, ny, nz], None

    def calculateNumberDensity(self, x, phi, rho, orbphase):
        x = np.asarray(x, dtype=np.float64)
        scalar = np.ndim(phi) == 0 and np.ndim(rho) == 0
        phi_, rho_ = np.broadcast_arrays(np.atleast_1d(phi), np.atleast_1d(rho))
        y, z = geom.Grid.getCartesianFromCylinder(phi_, rho_)
        px = np.broadcast_to(x[None, :], (len(y), len(x)))
        py = np.broadcast_to(np.asarray(y, dtype=np.float64)[:, None], px.shape)
        pz = np.broadcast_to(np.asarray(z, dtype=np.float64)[:, None], px.shape)
        self.checkBounds(px, py, pz)
        dev = _device()
        with dev.lock:
            n = dev.gridded_density(*self.gridAxes, self.gridValues, px, py, pz)
        return n[0] if scalar else n


# ============================================================================== cross sections
class AtmosphericConstituent:
    """Atom/ion absorber; its sigma(lambda) is a sum of Voigt lines from the NIST list
    (gasProperties.py:609-735).  The table is built on the GPU."""

    def __init__(self, species: Any, chi: float, sigma_v: float):
        self.isMolecule = False
        self.species = species
        self.chi = chi
        self.sigma_v = sigma_v
        self.wavelengthGridRefinement = 10.
        self.wavelengthGridExtension = 0.01
        self.lookupOffset = 1e-50

    def getLineParameters(self, wavelength) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Lines of this species strictly inside (min, max) of ``wavelength``: centre [cm],
        gamma = A/(4 pi), oscillator strength (gasProperties.py:640-670)."""
        ll = LINE_LIST
        mine = (ll[:, 0] == self.species.element) & (ll[:, 1] == self.species.ionizationState) & \
            (ll[:, 2] != '') & (ll[:, 3] != '') & (ll[:, 4] != '')
        lam = ll[mine, 2].astype(float) * 1e-8
        gam = ll[mine, 3].astype(float) / (4. * np.pi)
        f = ll[mine, 4].astype(float)
        inside = (lam > min(wavelength)) & (lam < max(wavelength))
        return lam[inside], gam[inside], f[inside]

    def _lines(self, wavelength):
        lam, gam, f = self.getLineParameters(wavelength)
        # (pi e^2 / (m_e c)) * f, evaluated left to right as in gasProperties.py:689-691
        coef = np.array([np.pi * const.e ** 2 / (const.m_e * const.c) * fi for fi in f], dtype=np.float64)
        return lam, gam, coef

    def calculateVoigtProfile(self, wavelength) -> np.ndarray:
        w = np.asarray(wavelength, dtype=np.float64)
        lam, gam, coef = self._lines(w)
        dev = _device()
        with dev.lock:
            return dev.voigt_sigma(w.ravel(), lam, gam, coef, self.sigma_v, const.c).reshape(w.shape)

    def constructLookupFunction(self, wavelengthGrid: "WavelengthGrid") -> LookupTable:
        refined = deepcopy(wavelengthGrid)
        refined.resolutionHigh /= self.wavelengthGridRefinement
        refined.lower_w *= (1. - self.wavelengthGridExtension)
        refined.upper_w *= (1. + self.wavelengthGridExtension)
        x = refined.constructWavelengthGridSingle(self)
        lam, gam, coef = self._lines(x)
        dev = _device()
        with dev.lock:
            tid, y = dev.table_build_voigt(x, lam, gam, coef, self.sigma_v, const.c, self.lookupOffset)
        return LookupTable(x, y, self.lookupOffset, {dev.device: tid})

    def addLookupFunctionToConstituent(self, wavelengthGrid: "WavelengthGrid") -> None:
        self.lookupFunction = self.constructLookupFunction(wavelengthGrid)

    def getSigmaAbs(self, wavelength) -> np.ndarray:
        w = np.asarray(wavelength, dtype=np.float64)
        dev = _device()
        with dev.lock:
            return dev.table_lookup(self.lookupFunction.table_id(dev), w.ravel()).reshape(w.shape)


class MolecularTable:
    """(P [dyn cm^-2], T [K], lambda [cm], log10(xsec + offset)) after the reference's conversions
    (gasProperties.py:774-781), with per-device uploaded copies."""

    def __init__(self, P, T, W, V, offset):
        self.P, self.T, self.W, self.V, self.offset = P, T, W, V, offset
        self.grid = (P, T, W)
        self._ids: Dict[int, int] = {}
        self._lock = threading.Lock()
        weakref.finalize(self, _release_tables, self._ids, True)

    def __deepcopy__(self, memo):
        return MolecularTable(*(deepcopy(a, memo) for a in (self.P, self.T, self.W, self.V)), self.offset)

    def table_id(self, dev) -> int:
        with self._lock:
            tid = self._ids.get(dev.device)
            if tid is None:
                tid = dev.molecular_upload(self.P, self.T, self.W, self.V, self.offset)
                self._ids[dev.device] = tid
            return tid


def _read_molecular_source(name: str) -> dict:
    if name in _MOLECULAR_TABLES:
        return _MOLECULAR_TABLES[name]
    base = os.path.join(molecularLookupPath, name)
    if os.path.exists(base + ".npz"):
        with np.load(base + ".npz", allow_pickle=False) as d:
            return {k: d[k] for k in ("p", "t", "bin_edges", "xsecarr")}
    if os.path.exists(base + ".h5"):
        import h5py  # optional dependency, as in the reference
        with h5py.File(base + ".h5", "r") as f:
            return {k: f[k][:] for k in ("p", "t", "bin_edges", "xsecarr")}
    raise FileNotFoundError("no molecular table %r (register_molecular_table, %s.npz or %s.h5)" % (name, base, base))


class MolecularConstituent:
    """Molecule with a (P, T, lambda) cross-section table (gasProperties.py:738-818)."""

    def __init__(self, moleculeName: str, chi: float):
        self.isMolecule = True
        self.lookupOffset = 1e-50
        self.moleculeName = moleculeName
        self.chi = chi

    def constructLookupFunction(self) -> MolecularTable:
        src = _read_molecular_source(self.moleculeName)
        P = np.asarray(src["p"], dtype=np.float64) * 10.
        T = np.asarray(src["t"], dtype=np.float64)
        W = 1. / np.asarray(src["bin_edges"], dtype=np.float64)[::-1]
        V = np.log10(np.asarray(src["xsecarr"], dtype=np.float64)[:, :, ::-1] + self.lookupOffset)
        return MolecularTable(P, T, np.ascontiguousarray(W), np.ascontiguousarray(V), self.lookupOffset)

    def addLookupFunctionToConstituent(self) -> None:
        self.lookupFunction = self.constructLookupFunction()

    def getSigmaAbs(self, P, T, wavelength) -> np.ndarray:
        dev = _device()
        with dev.lock:
            return dev.molecular_sigma(self.lookupFunction.table_id(dev), np.asarray(P, np.float64), T,
                                       np.asarray(wavelength, np.float64))


# ============================================================================== atmosphere
class Atmosphere:
    """All density distributions of a run (gasProperties.py:821-956)."""

    def __init__(self, densityDistributionList: List[Any], hasOrbitalDopplerShift: bool):
        self.densityDistributionList = densityDistributionList
        self.hasOrbitalDopplerShift = hasOrbitalDopplerShift

    @staticmethod
    def getAbsorberNumberDensity(densityDistribution, chi, x, phi, rho, orbphase):
        return densityDistribution.calculateNumberDensity(x, phi, rho, orbphase) * chi

    def getAbsorberVelocityField(self, densityDistribution, x, phi, rho, orbphase):
        v = np.zeros_like(x)
        if self.hasOrbitalDopplerShift:
            body = densityDistribution.moon if densityDistribution.hasMoon else densityDistribution.planet
            v += body.getLOSvelocity(orbphase)
        return v

    def shifts(self, densityDistribution, orbphase) -> np.ndarray:
        """Per-phase Doppler factor of one distribution (gasProperties.py:907-917)."""
        orbphase = np.asarray(orbphase, dtype=np.float64)
        if self.hasOrbitalDopplerShift:
            body = densityDistribution.moon if densityDistribution.hasMoon else densityDistribution.planet
            v = body.getLOSvelocity(orbphase)
        else:
            v = np.zeros(len(orbphase))
        return const.calculateDopplerShift(-v)


# ============================================================================== wavelength grid
class WavelengthGrid:
    """Non-uniform wavelength grid: resolutionHigh inside windows of width widthHighRes around each
    line, resolutionLow elsewhere (gasProperties.py:959-1071).  Node generation keeps the
    reference's sequence of numpy ``arange`` calls, which fixes every node to the bit."""

    def __init__(self, lower_w: float, upper_w: float, widthHighRes: float, resolutionLow: float,
                 resolutionHigh: float):
        self.lower_w = lower_w
        self.upper_w = upper_w
        self.widthHighRes = widthHighRes
        self.resolutionLow = resolutionLow
        self.resolutionHigh = resolutionHigh

    def arangeWavelengthGrid(self, linesList) -> np.ndarray:
        peaks = np.sort(np.unique(linesList))
        if len(peaks) == 0:
            print('WARNING: No absorption lines from atoms/ions in the specified wavelength range!')
            return np.arange(self.lower_w, self.upper_w, self.resolutionLow)
        w = self.widthHighRes
        gaps = np.concatenate(([np.inf], np.diff(peaks), [np.inf]))
        lo_edges = [p - w / 2. for i, p in enumerate(peaks) if gaps[i] > w]
        hi_edges = [p + w / 2. for i, p in enumerate(peaks) if gaps[i + 1] > w]
        segs = []
        last = len(lo_edges) - 1
        for i in range(len(lo_edges)):
            segs.append(np.arange(lo_edges[i], hi_edges[i], self.resolutionHigh))
            if i == 0:
                if self.lower_w < lo_edges[0]:
                    segs.append(np.arange(self.lower_w, lo_edges[0], self.resolutionLow))
                if last == 0 and self.upper_w > hi_edges[-1]:
                    segs.append(np.arange(hi_edges[0], self.upper_w, self.resolutionLow))
                continue
            segs.append(np.arange(hi_edges[i - 1], lo_edges[i], self.resolutionLow))
            if i == last and self.upper_w > hi_edges[-1]:
                segs.append(np.arange(hi_edges[-1], self.upper_w, self.resolutionLow))
        return np.sort(np.concatenate(segs))

    def constructWavelengthGridSingle(self, constituent: AtmosphericConstituent) -> np.ndarray:
        return self.arangeWavelengthGrid(constituent.getLineParameters(np.array([self.lower_w, self.upper_w]))[0])

    def constructWavelengthGrid(self, densityDistributionList: List[Any]) -> np.ndarray:
        lines: List[float] = []
        for dist in densityDistributionList:
            for con in dist.constituents:
                if not con.isMolecule:
                    lines.extend(con.getLineParameters(np.array([self.lower_w, self.upper_w]))[0])
        if len(lines) == 0:
            return np.arange(self.lower_w, self.upper_w, self.resolutionLow)
        return self.arangeWavelengthGrid(lines)


# ============================================================================== transit
_STAR_TABLES: "weakref.WeakKeyDictionary" = None


def _star_lookup_table(fn) -> "LookupTable":
    """Device copies of an Fstar_function's (x, log10 F) (offset 0: n_interp_log(..., 0.0),
    gasProperties.py:1212-1219; 10**Fstar_function(...), celestialBodies.py:239), kept per function object."""
    global _STAR_TABLES
    import weakref
    if isinstance(fn, LookupTable):
        return fn
    if _STAR_TABLES is None:
        _STAR_TABLES = weakref.WeakKeyDictionary()
    x = np.ascontiguousarray(np.asarray(fn.x, dtype=np.float64))
    y = np.ascontiguousarray(np.asarray(fn.y, dtype=np.float64))
    # the cached device copy stays valid only while the spectrum's content is unchanged (arrays replaced or
    # modified in place): a content fingerprint of both arrays is part of the key
    fp = _content_fingerprint(x, y)
    try:
        hit = _STAR_TABLES.get(fn)
    except TypeError:   # not weak-referenceable: no cache
        hit = None
    if hit is not None and hit[1] == fp:
        return hit[0]
    if np.any(x[1:] < x[:-1]):
        raise ValueError("Fstar_function.x must be ascending (np.interp, gasProperties.py:1214)")
    tab = LookupTable(x, y, 0.0)
    try:
        _STAR_TABLES[fn] = (tab, fp)
    except TypeError:
        pass
    return tab


def _content_fingerprint(*arrays) -> tuple:
    """(shape, 64-bit content hash) per array: xxhash's xxh3_64 when importable, else blake2b with an 8-byte
    digest."""
    try:
        import xxhash

        def h(b):
            return xxhash.xxh3_64_intdigest(b)
    except ImportError:   # pragma: no cover
        import hashlib

        def h(b):
            return hashlib.blake2b(b, digest_size=8).digest()
    return tuple((a.shape, h(memoryview(a).cast("B"))) for a in arrays)


class Transit:
    """Transit depth R(orbital phase, wavelength) (gasProperties.py:1074-1258)."""

    def __init__(self, atmosphere: Atmosphere, wavelengthGrid: WavelengthGrid, spatialGrid: geom.Grid):
        self.atmosphere = atmosphere
        self.wavelengthGrid = wavelengthGrid
        self.spatialGrid = spatialGrid
        self.planet = self.atmosphere.densityDistributionList[0].planet
        self.last_stats: List[dict] = []
        # per-run device statistics in last_stats (stage times, chord counts, exp evaluations): they time
        # the run with events and count in the kernels, ~0.1 ms per call, so off unless asked for
        # (this attribute, or PROM_COLLECT_STATS=1 in the environment)
        self.collect_stats = os.environ.get("PROM_COLLECT_STATS", "0") not in ("", "0")

    def addWavelength(self) -> None:
        # page-locked copy (_native.pinned_copy): the grid is sent to the device on every call
        self.wavelength = _native.pinned_copy(
            self.wavelengthGrid.constructWavelengthGrid(self.atmosphere.densityDistributionList))

    def checkBlock(self, phi: float, rho: float, orbphase: float) -> bool:
        """Scalar blocking test (gasProperties.py:1107-1130; the moon test uses R_moon^2 here,
        as the batched path does, not R_moon)."""
        y, z = geom.Grid.getCartesianFromCylinder(phi, rho)
        if np.sqrt((y - self.planet.getPosition(orbphase)[1]) ** 2 + z ** 2) < self.planet.R:
            return True
        for d in self.atmosphere.densityDistributionList:
            if d.hasMoon and (y - d.moon.getPosition(orbphase)[1]) ** 2 + z ** 2 < d.moon.R ** 2:
                return True
        return False

    # ---- host-side set-up: O(n_phase + n_chord-positions) scalars, numpy as in the reference ----
    def _chord_geometry(self, g, star) -> tuple:
        """(phi, rho, y, z, clv, fout, orbphase, x) of the chord grid: a function of the grid's and the
        star's scalars only, so it is kept and rebuilt when any of them changes (retrieval loops call
        sumOverChords with the same geometry and new densities)."""
        key = (g.x_midpoint, g.x_border, g.x_steps, g.rho_border, g.rho_steps, g.phi_steps, g.orbphase_border,
               g.orbphase_steps, star.R, star.CLV_u1, star.CLV_u2)
        cached = getattr(self, "_geo_cache", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        phi, rho = g.getChordPositions()
        y, z = rho * np.sin(phi), rho * np.cos(phi)
        mu = np.sqrt(np.clip(1. - rho ** 2 / star.R ** 2, 0, 1))
        clv = 1. - star.CLV_u1 * (1. - mu) - star.CLV_u2 * (1. - mu) ** 2
        fout = rho * (np.ones_like(clv) * clv)
        geo = (phi, rho, y, z, clv, fout, g.constructOrbphaseAxis(), g.constructXaxis())
        for a in geo:
            a.flags.writeable = False
        self._geo_cache = (key, geo)
        return geo

    def _host_inputs(self) -> dict:
        g = self.spatialGrid
        star = self.planet.hostStar
        phi, rho, y, z, clv, fout, orb, xaxis = self._chord_geometry(g, star)
        stellar = None
        if star.Fstar_function is not None:
            # gasProperties.py:1183-1184: the Rossiter-McLaughlin shift of each chord's stellar spectrum
            v_star = star.vsiniStarrot * rho / star.R * np.cos(phi - star.phiStarrot)
            stellar = {"rho": rho, "clv": clv, "shift": const.calculateDopplerShift(v_star),
                       "table": self._star_table(star.Fstar_function)}
        moons = [d.moon for d in self.atmosphere.densityDistributionList if d.hasMoon]
        scen = []
        need_tab = []
        for d in self.atmosphere.densityDistributionList:
            entry = {"dist": d, "shift": self.atmosphere.shifts(d, orb), "T": float(getattr(d, "T", 0.0) or 0.0)}
            try:
                kind, params, body = d.densityModel()
                if kind == _native.DENSITY_GRIDDED:
                    d.checkBounds(xaxis[None, :], y[:, None], z[:, None])
                    entry.update(kind=kind, params=params, n_tabulated=d._packed)
                else:
                    bx, by = body.getPosition(orb)
                    entry.update(kind=kind, params=params, body_x=np.asarray(bx, float),
                                 body_y=np.asarray(by, float))
            except NotImplementedError:
                entry.update(kind=_native.DENSITY_TABULATED, params=[])
                need_tab.append(entry)
            scen.append(entry)
        if need_tab:
            cg = g.getChordGrid()
            x = g.constructXaxis()
            for e in need_tab:
                e["n_tabulated"] = np.asarray(e["dist"].calculateNumberDensity(x, cg[:, 0], cg[:, 1], cg[:, 2]),
                                              dtype=np.float64).reshape(len(cg), len(x))
        return {"y": y, "z": z, "fout": fout, "orb": orb, "x": xaxis, "dx": g.getDeltaX(),
                "planet_y": self.planet.a * np.sin(orb), "planet_R": self.planet.R,
                "moon_y": np.array([m.getPosition(orb)[1] for m in moons]).reshape(len(moons), len(orb)),
                "moon_R": np.array([m.R for m in moons], dtype=np.float64), "scenarios": scen,
                "stellar": stellar}

    def _star_table(self, fn) -> "LookupTable":
        return _star_lookup_table(fn)

    def _problem(self, dev, host: dict, w0: int, w1: int, cull_tau: float,
                 options: int = 0) -> "_native.TransitInputs":
        star = None
        if host.get("stellar") is not None:
            st = host["stellar"]
            star = {"table_id": st["table"].table_id(dev), "rho": st["rho"], "clv": st["clv"], "shift": st["shift"]}
        scs = []
        for e in host["scenarios"]:
            cons = []
            for con in e["dist"].constituents:
                cons.append({"table_id": con.lookupFunction.table_id(dev), "is_molecule": con.isMolecule,
                             "chi": con.chi})
            scs.append({"kind": e["kind"], "params": e["params"], "body_x": e.get("body_x"),
                        "body_y": e.get("body_y"), "shift": e["shift"], "n_tabulated": e.get("n_tabulated"),
                        "T": e["T"], "constituents": cons})
        return _native.TransitInputs(
            wavelength=self.wavelength[w0:w1], chord_y=host["y"], chord_z=host["z"], chord_fout=host["fout"],
            n_orb=len(host["orb"]), x=host["x"], delta_x=host["dx"], planet_y=host["planet_y"],
            planet_R=host["planet_R"], moon_y=host["moon_y"], moon_R=host["moon_R"], scenarios=scs,
            cull_tau=cull_tau, options=options, k_B=const.k_B, star=star)

    def sumOverChords(self, max_memory_gb: float = 2.0, devices: Optional[Sequence[int]] = None,
                      cull_tau: float = 0.0, options: int = 0) -> np.ndarray:
        """R[n_orb, n_wav] = sum_chords F_out exp(-tau) / sum_chords F_out, on the GPU(s).

        ``devices``: GPU ids to shard the wavelength axis over (default: all visible GPUs when
        there are >= 65,536 wavelengths per GPU, else GPU 0).  ``max_memory_gb`` bounds the
        device working set of one shard step; larger shards are processed in several steps."""
        return self._integrate(max_memory_gb, devices, cull_tau, options, None)[0]

    def bandLightcurve(self, line_centers: Sequence[float] = None, bandwidth: float = None,
                       shifts=None, max_memory_gb: float = 2.0, devices: Optional[Sequence[int]] = None,
                       cull_tau: float = 0.0, options: int = 0, return_spectrum: bool = False):
        """Light curve: per phase, the mean of R over windows of ``bandwidth`` about the Doppler-shifted
        ``line_centers`` divided by the maximum of R (mainRetrieval.py:76-93; defaults Na D2/D1 and
        0.75 A, shifted by the planet's line-of-sight velocity).  The band reduction runs on the device
        over R in HBM; with ``return_spectrum`` R is copied back as well.  Returns the light curve
        [n_orb] (and R)."""
        from . import lightcurve as lc
        if not hasattr(self, "wavelength"):
            self.addWavelength()
        orb = self.spatialGrid.constructOrbphaseAxis()
        if shifts is None:
            shifts = lc.planet_shifts(self.planet, orb)
        bounds = lc.band_bounds(shifts, (lc.NA_D2, lc.NA_D1) if line_centers is None else line_centers,
                                lc.BANDWIDTH if bandwidth is None else bandwidth)
        R, acc = self._integrate(max_memory_gb, devices, cull_tau, options, bounds, want_R=return_spectrum)
        return (acc.lightcurve(), R) if return_spectrum else acc.lightcurve()

    def _integrate(self, max_memory_gb, devices, cull_tau, options, bounds, want_R=True):
        if not hasattr(self, "wavelength"):
            self.addWavelength()
        host = self._host_inputs()
        n_wav, n_orb = len(self.wavelength), len(host["orb"])
        if devices is None:
            avail = _native.device_count()
            if avail == 0:
                raise _native.NativeUnavailable("no HIP device visible")
            devices = list(range(min(avail, max(1, n_wav // 65536))))
        devices = list(devices)
        n_atoms = sum(1 for d in self.atmosphere.densityDistributionList for c in d.constituents
                      if not c.isMolecule)
        per_wav = 8 * n_orb * (2 + max(1, n_atoms))
        chunk = max(4096, int(max_memory_gb * 1e9) // per_wav) // WAVE_ALIGN * WAVE_ALIGN
        R = None
        if want_R:
            # one chunk on one device: R lands in page-locked memory from the library's pool in one DMA
            # (transit_result(out=R) below); otherwise (or past the pool's cap) ordinary memory
            if len(devices) == 1 and n_wav <= chunk:
                R = _native.host_array((n_orb, n_wav))
            if R is None:
                R = np.empty((n_orb, n_wav))
        acc = None
        if bounds is not None:
            from .lightcurve import BandAccumulator
            acc = BandAccumulator(n_orb)
        acc_lock = threading.Lock()
        shards = _split(n_wav, len(devices))
        errors: List[BaseException] = []
        self.last_stats = []

        def work(dev_id: int, lo: int, hi: int):
            try:
                dev = _native.get_device(dev_id)
                with dev.lock:
                    for a in range(lo, hi, chunk):
                        b = min(hi, a + chunk)
                        dev.transit_set(self._problem(dev, host, a, b, cull_tau, options))
                        st = dev.transit_run(stats=True) if self.collect_stats else dev.transit_run() or {}
                        if R is not None:
                            if a == 0 and b == n_wav:   # one chunk: straight into the result
                                dev.transit_result(out=R)
                            else:
                                R[:, a:b] = dev.transit_result()
                        if acc is not None:
                            part = dev.transit_band_stats(bounds)
                            with acc_lock:
                                acc.add(*part)
                        st.update(device=dev_id, w0=a, w1=b)
                        self.last_stats.append(st)
            except BaseException as ex:  # re-raised in the caller
                errors.append(ex)

        if len(shards) == 1:
            work(devices[0], *shards[0])
        else:
            th = [threading.Thread(target=work, args=(devices[i], a, b)) for i, (a, b) in enumerate(shards)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        if errors:
            raise errors[0]
        return R, acc
