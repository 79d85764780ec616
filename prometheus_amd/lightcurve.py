"""Band-averaged light curves of a transit spectrum (the post-processing of mainRetrieval.py:76-93).

For each orbital phase o the reference averages R(o, lambda) over the wavelengths inside windows of
width ``bandwidth`` centred on Doppler-shifted line centres (Na D2 and D1 by default, shifted by the
planet's line-of-sight velocity at that phase) and divides by the maximum of R(o, :).  Here the
reduction runs on the device over R as it stays in HBM after the run (prom_transit_band_stats); the
host only forms the O(n_phase) window bounds and combines the per-shard partial sums.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from . import constants as const

NA_D2 = 5891.583253e-8   # cm (mainRetrieval.py:83)
NA_D1 = 5897.558147e-8   # cm (mainRetrieval.py:84)
BANDWIDTH = 0.75e-8      # cm (mainRetrieval.py:79)


def band_bounds(shift, centers: Sequence[float] = (NA_D2, NA_D1), bandwidth: float = BANDWIDTH) -> np.ndarray:
    """[n_orb][n_bands][2] window limits (centre * shift - bandwidth / 2, centre * shift + bandwidth / 2),
    inclusive at both ends, in the reference's evaluation order."""
    shift = np.atleast_1d(np.asarray(shift, dtype=np.float64))
    out = np.empty((len(shift), len(centers), 2))
    for b, c in enumerate(centers):
        out[:, b, 0] = c * shift - bandwidth / 2.
        out[:, b, 1] = c * shift + bandwidth / 2.
    return out


def planet_shifts(planet, orbphase) -> np.ndarray:
    """Doppler factors of the planet's line-of-sight velocity per phase (mainRetrieval.py:80-81)."""
    return const.calculateDopplerShift(planet.getLOSvelocity(np.asarray(orbphase, dtype=np.float64)))


class BandAccumulator:
    """Combines prom_transit_band_stats partials over wavelength shards / chunks."""

    def __init__(self, n_orb: int) -> None:
        self.sum = np.zeros(n_orb)
        self.count = np.zeros(n_orb, dtype=np.int64)
        self.max = np.full(n_orb, -np.inf)

    def add(self, s, c, m) -> None:
        self.sum += s
        self.count += c
        nan = np.isnan(self.max) | np.isnan(m)
        self.max = np.where(nan, np.nan, np.maximum(self.max, m))

    def lightcurve(self) -> np.ndarray:
        with np.errstate(invalid="ignore", divide="ignore"):
            mean = np.where(self.count > 0, self.sum / np.maximum(self.count, 1), np.nan)
            return mean / self.max
