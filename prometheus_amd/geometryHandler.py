"""Spatial/temporal grid of the transit integrator (mirrors ``pythonScripts/geometryHandler.py``).

Observer at x = -inf, star at the origin, sky plane (y, z) with polar coordinates
(rho, phi).  Chords are the (phi, rho) cell midpoints; each is integrated along x with
``x_steps`` midpoint samples.  Axes use numpy ``linspace`` exactly like the reference so
that every node is bit-identical.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


class Grid:
    def __init__(self, x_midpoint: float, x_border: float, x_steps: int, rho_border: float, rho_steps: int,
                 phi_steps: int, orbphase_border: float, orbphase_steps: int) -> None:
        self.x_midpoint = x_midpoint
        self.x_border = x_border
        self.x_steps = x_steps
        self.rho_border = rho_border
        self.rho_steps = rho_steps
        self.phi_steps = phi_steps
        self.orbphase_border = orbphase_border
        self.orbphase_steps = orbphase_steps

    @staticmethod
    def getCartesianFromCylinder(phi, rho) -> Tuple:
        """(y, z) = rho (sin phi, cos phi)   (geometryHandler.py:73-86)."""
        return rho * np.sin(phi), rho * np.cos(phi)

    def getDeltaX(self) -> float:
        return 2. * self.x_border / float(self.x_steps)

    def getDeltaRho(self) -> float:
        return self.rho_border / float(self.rho_steps)

    def getDeltaPhi(self) -> float:
        return 2. * np.pi / float(self.phi_steps)

    def constructXaxis(self, midpoints: bool = True) -> np.ndarray:
        lo, hi, n = self.x_midpoint - self.x_border, self.x_midpoint + self.x_border, int(self.x_steps)
        if midpoints:
            return np.linspace(lo, hi, n, endpoint=False) + self.x_border / float(self.x_steps)
        return np.linspace(lo, hi, n + 1)

    def constructRhoAxis(self, midpoints: bool = True) -> np.ndarray:
        n = int(self.rho_steps)
        if midpoints:
            return np.linspace(0., self.rho_border, n, endpoint=False) + 0.5 * self.rho_border / float(self.rho_steps)
        return np.linspace(0., self.rho_border, n + 1)

    def constructPhiAxis(self, midpoints: bool = True) -> np.ndarray:
        n = int(self.phi_steps)
        if midpoints:
            return np.linspace(0, 2 * np.pi, n, endpoint=False) + np.pi / float(self.phi_steps)
        return np.linspace(0, 2 * np.pi, n + 1)

    def constructOrbphaseAxis(self) -> np.ndarray:
        return np.linspace(-self.orbphase_border, self.orbphase_border, int(self.orbphase_steps))

    def getChordPositions(self) -> Tuple[np.ndarray, np.ndarray]:
        """(phi, rho) of the n_phi*n_rho chord positions, phi-major (the chord grid without phase)."""
        P, R = np.meshgrid(self.constructPhiAxis(), self.constructRhoAxis(), indexing="ij")
        return P.ravel(), R.ravel()

    def getChordGrid(self) -> np.ndarray:
        """All (phi, rho, orbphase) triples, orbital phase fastest (geometryHandler.py:188-208)."""
        P, R, O = np.meshgrid(self.constructPhiAxis(), self.constructRhoAxis(), self.constructOrbphaseAxis(),
                              indexing="ij")
        return np.stack((P.ravel(), R.ravel(), O.ravel()), axis=-1)
