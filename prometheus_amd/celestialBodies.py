"""Star, planet, moon and the bundled system catalogue (mirrors ``pythonScripts/celestialBodies.py``).

Orbital geometry is evaluated on the host with numpy: it is O(n_orbphase) scalar work (positions
and line-of-sight velocities per phase) that feeds the device kernels, and keeping numpy here makes
those per-phase scalars bit-identical to the reference.  The O(chords x samples) distance fields
(``getDistanceFromPlanet`` etc.) are kept for user-written density plugins; the built-in scenarios
evaluate them on the GPU instead (``prom_number_density`` / the fused transit kernel).
"""
from __future__ import annotations

import csv
import os
from typing import Any, Optional, Tuple

import numpy as np

from . import constants as const
from . import geometryHandler as geom

_RES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resources")


class Star:
    """Host star: radius/mass [cgs], CLV coefficients, rotation (celestialBodies.py:26-95)."""

    def __init__(self, R: float, dR: float, M: float, dM: float, T_eff: float, dT_eff: float, log_g: float,
                 dlog_g: float, Z: float, dZ: float, alpha: float) -> None:
        self.R, self.dR, self.M, self.dM = R, dR, M, dM
        self.T_eff, self.dT_eff, self.log_g, self.dlog_g = T_eff, dT_eff, log_g, dlog_g
        self.Z, self.dZ, self.alpha = Z, dZ, alpha
        self.CLV_u1 = 0.
        self.CLV_u2 = 0.
        self.vsiniStarrot = 0.
        self.phiStarrot = 0.
        self.Fstar_function = None

    def addCLVparameters(self, CLV_u1: float, CLV_u2: float) -> None:
        self.CLV_u1, self.CLV_u2 = CLV_u1, CLV_u2

    def addRMparameters(self, vsiniStarrot: float, phiStarrot: float) -> None:
        self.vsiniStarrot, self.phiStarrot = vsiniStarrot, phiStarrot

    def getSurfaceVelocity(self, phi, rho):
        return self.vsiniStarrot * rho / self.R * np.cos(phi - self.phiStarrot)

    @staticmethod
    def round_to_grid(grid, value):
        """The grid point closest to value, the first one on a tie (celestialBodies.py:113-126)."""
        diff = np.subtract(value, grid)
        return grid[np.argmin(np.abs(diff))]

    def calculateCLV(self, rho):
        arg = 1. - np.sqrt(1. - rho ** 2 / self.R ** 2)
        return 1. - self.CLV_u1 * arg - self.CLV_u2 * arg ** 2

    def calculateRM(self, phi, rho, wavelength):
        """Stellar flux of the surface point (phi, rho), Doppler-shifted by the star's rotation:
        10**Fstar_function(wavelength / shift) (celestialBodies.py:226-240).  O(n_wavelength) for one
        point, as in the reference; the disk integral runs on the GPU (getFstarIntegrated)."""
        shift = const.calculateDopplerShift(self.getSurfaceVelocity(phi, rho))
        return 10. ** self.Fstar_function(wavelength / shift)

    def getFstar(self, phi, rho, wavelength):
        """Flux of one disk point: CLV only without rotation, else calculateRM * CLV
        (celestialBodies.py:313-332)."""
        if self.vsiniStarrot == 0.:
            return np.ones_like(wavelength) * self.calculateCLV(rho)
        Fstar = self.calculateRM(phi, rho, wavelength)
        Fstar *= self.calculateCLV(rho)
        return Fstar

    def getFstarIntegrated(self, wavelength, grid, device: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
        """(disk-integrated flux, flux of the disk outside rho_border) (celestialBodies.py:267-311).

        Without rotation both are the reference's closed forms (scalars broadcast over the wavelengths).
        With rotation the disk integral sum_phi sum_rho F(lambda / s) clv dphi drho rho over the grid's
        cells runs on the GPU (prom_star_disk_flux; the per-cell Doppler and CLV factors are formed here
        exactly as the reference forms them), and the second value is zeros, as in the reference."""
        if self.vsiniStarrot == 0.:
            FstarIntegrated = np.pi * self.R ** 2 * (1. - self.CLV_u1 / 3. - self.CLV_u2 / 6.) * \
                np.ones_like(wavelength)
            upperTerm = 0.5 * (-self.CLV_u2 * self.R ** 2 - self.CLV_u1 * self.R ** 2 + self.R ** 2)
            rb = grid.rho_border
            term1 = -4. * self.R ** 2 * self.CLV_u1 * (1. - rb ** 2 / self.R ** 2) ** 1.5
            term2 = self.R ** 2 * self.CLV_u2 * (6 * rb ** 2 / self.R ** 2 + 8. * (1. - rb ** 2 / self.R ** 2) ** 1.5 -
                                                 3. * (self.R ** 2 - rb ** 2) ** 2 / self.R ** 4)
            lowerTerm = 1. / 12. * (term1 - term2 - 6. * self.CLV_u1 * rb ** 2 + 6. * rb ** 2)
            FstarUpper = 2. * np.pi * (upperTerm - lowerTerm) * np.ones_like(wavelength)
            return FstarIntegrated, FstarUpper
        from . import _native
        from .gasProperties import _star_lookup_table
        phiArray, rhoArray = grid.constructPhiAxis(), grid.constructRhoAxis()
        if len(phiArray) == 0 or len(rhoArray) == 0:
            raise UnboundLocalError("getFstarIntegrated: empty disk grid (the reference's FstarUpper is unset)")
        shift, clv, rho = [], [], []
        for phi in phiArray:          # the reference's loop order: phi outer, rho inner
            for r in rhoArray:
                shift.append(const.calculateDopplerShift(self.getSurfaceVelocity(phi, r)))
                clv.append(self.calculateCLV(r))
                rho.append(r)
        w = np.asarray(wavelength, dtype=np.float64)
        dev = _native.get_device(_native.default_device() if device is None else device)
        tab = _star_lookup_table(self.Fstar_function)
        with dev.lock:
            out = dev.star_disk_flux(tab.table_id(dev), shift, clv, rho, grid.getDeltaPhi(), grid.getDeltaRho(),
                                     w.ravel())
        return out.reshape(w.shape), np.zeros_like(w)

    def getSpectrum(self):
        raise NotImplementedError("PHOENIX spectra are fetched over FTP by the reference "
                                  "(celestialBodies.py:128-209); this build has no network: provide the "
                                  "spectrum with addFstarSpectrum(wavelength, flux) or set Fstar_function")

    def addFstarFunction(self, wavelength) -> None:
        self.getSpectrum()

    def addFstarSpectrum(self, wavelength, flux) -> None:
        """Fstar_function from a spectrum already at hand: the reference keeps
        interp1d(w_starSEL, log10(F_0)) (celestialBodies.py:223-235) and reads only its .x / .y
        (gasProperties.py:1212-1219); wavelength [cm] ascending, flux > 0 in any unit (R is a ratio)."""
        w = np.asarray(wavelength, dtype=np.float64)
        order = np.argsort(w, kind="mergesort")   # interp1d sorts its x the same way
        self.Fstar_function = StellarSpectrum(w[order], np.log10(np.asarray(flux, dtype=np.float64))[order])


class StellarSpectrum:
    """(x, y = log10 F) pair standing in for the reference's interp1d (only .x and .y are read)."""

    def __init__(self, x, y) -> None:
        self.x = np.ascontiguousarray(x, dtype=np.float64)
        self.y = np.ascontiguousarray(y, dtype=np.float64)

    def __call__(self, w):
        """interp1d(x, y, kind='linear') evaluation: numpy.interp inside [x_0, x_{n-1}], ValueError outside
        (bounds_error, scipy's default for the reference's Fstar_function)."""
        w = np.asarray(w, dtype=np.float64)
        if np.any(w < self.x[0]):
            raise ValueError("A value in x_new is below the interpolation range's minimum value (%r)." % self.x[0])
        if np.any(w > self.x[-1]):
            raise ValueError("A value in x_new is above the interpolation range's maximum value (%r)." % self.x[-1])
        return np.interp(w, self.x, self.y)


class Planet:
    """Planet on a circular, edge-on orbit (celestialBodies.py:335-470)."""

    def __init__(self, name: str, R: float, M: float, a: float, hostStar: Star, transitDuration: float,
                 orbitalPeriod: float, b: float) -> None:
        self.name, self.R, self.M, self.a, self.hostStar = name, R, M, a, hostStar
        self.transitDuration, self.orbitalPeriod, self.b = transitDuration, orbitalPeriod, b

    def getPosition(self, orbphase) -> Tuple[Any, Any]:
        return self.a * np.cos(orbphase), self.a * np.sin(orbphase)

    def getLOSvelocity(self, orbphase):
        return -np.sin(orbphase) * np.sqrt(const.G * self.hostStar.M / self.a)

    def getDistanceFromPlanet(self, x, phi, rho, orbphase):
        y, z = geom.Grid.getCartesianFromCylinder(phi, rho)
        xp, yp = self.getPosition(orbphase)
        x_, xp_, yp_, y_, z_ = _batch(x, xp, yp, y, z)
        return np.sqrt((x_ - xp_) ** 2 + (y_ - yp_) ** 2 + z_ ** 2)

    def getTorusCoords(self, x, phi, rho, orbphase):
        y, z = geom.Grid.getCartesianFromCylinder(phi, rho)
        xp, yp = self.getPosition(orbphase)
        x_, xp_, yp_, y_, z_ = _batch(x, xp, yp, y, z)
        return np.sqrt((x_ - xp_) ** 2 + (y_ - yp_) ** 2), z_


class Moon:
    """Moon on a circular orbit around its planet (celestialBodies.py:473-583)."""

    def __init__(self, midTransitOrbphase: float, R: float, a: float, hostPlanet: Planet) -> None:
        self.midTransitOrbphase, self.R, self.a, self.hostPlanet = midTransitOrbphase, R, a, hostPlanet

    def getOrbphase(self, orbphase):
        p = self.hostPlanet
        ratio = np.sqrt((np.float64(p.a) ** 3 * np.float64(p.M)) /
                        (np.float64(self.a) ** 3 * np.float64(p.hostStar.M)))
        return self.midTransitOrbphase + np.float64(orbphase) * ratio

    def getPosition(self, orbphase):
        om = self.getOrbphase(orbphase)
        xp, yp = self.hostPlanet.getPosition(orbphase)
        return xp + self.a * np.cos(om), yp + self.a * np.sin(om)

    def getLOSvelocity(self, orbphase):
        vp = self.hostPlanet.getLOSvelocity(orbphase)
        return vp - np.sin(self.getOrbphase(orbphase)) * np.sqrt(const.G * self.hostPlanet.M / self.a)

    def getDistanceFromMoon(self, x, phi, rho, orbphase):
        y, z = geom.Grid.getCartesianFromCylinder(phi, rho)
        xm, ym = self.getPosition(orbphase)
        x_, xm_, ym_, y_, z_ = _batch(x, xm, ym, y, z)
        return np.sqrt((x_ - xm_) ** 2 + (y_ - ym_) ** 2 + z_ ** 2)


def _batch(x, bx, by, y, z):
    """Scalar chord -> (n_x,); arrays of chords -> (n_chords, n_x) (celestialBodies.py:421-435)."""
    x, bx, by, y, z = (np.asarray(v) for v in (x, bx, by, y, z))
    if bx.ndim > 0:
        return x[np.newaxis, :], bx[:, np.newaxis], by[:, np.newaxis], y[:, np.newaxis], z[:, np.newaxis]
    return x, bx, by, y, z


class AvailablePlanets:
    """Systems from the bundled ``resources/stars.csv`` and ``planets.csv`` (celestialBodies.py:586-664)."""

    def __init__(self) -> None:
        self.stars = {}
        with open(os.path.join(_RES, "stars.csv"), newline="") as fh:
            for row in csv.DictReader(fh):
                f = {k: float(v) for k, v in row.items() if k != "name"}
                self.stars[row["name"]] = Star(f["R_sun"] * const.R_sun, f["dR_sun"] * const.R_sun,
                                               f["M_sun"] * const.M_sun, f["dM_sun"] * const.M_sun, f["T_eff"],
                                               f["dT_eff"], f["log_g"], f["dlog_g"], f["Fe_H"], f["dFe_H"], 0)
        self.planetList = []
        with open(os.path.join(_RES, "planets.csv"), newline="") as fh:
            for row in csv.DictReader(fh):
                star = self.stars.get(row["hostStar"])
                if star is None:
                    print(f"Warning: Host star {row['hostStar']} not found for planet {row['name']}")
                    continue
                self.planetList.append(Planet(row["name"], float(row["R_J"]) * const.R_J,
                                              float(row["M_J"]) * const.M_J, float(row["a_AU"]) * const.AU, star,
                                              float(row["transitDuration"]), float(row["P"]),
                                              float(row["b"]) * star.R))

    def listPlanetNames(self):
        return [p.name for p in self.planetList]

    def findPlanet(self, namePlanet: str) -> Optional[Planet]:
        for p in self.planetList:
            if p.name == namePlanet:
                return p
        print('System', namePlanet, 'was not found.')
        return None
