"""cgs constants, the relativistic Doppler factor and the species table.

Mirrors ``pythonScripts/constants.py`` (same names, same numerical values: the
reference's own rounded constants are kept, not CODATA, because R depends on them).
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

# constants.py:13-26 -- expressions kept as written so every float is bit-identical
e = 4.803e-10
m_e = 9.109e-28
c = 2.998e10
G = 6.674 * 10 ** (-8)
k_B = 1.381 * 10 ** (-16)
amu = 1.661 * 10 ** (-24)
R_J = 7.1492e9
M_J = 1.898e30
M_E = 5.974e27
R_sun = 6.96e10
M_sun = 1.988e33
R_Io = 1.822e8
euler_mascheroni = 0.57721
AU = 1.496e13


def calculateDopplerShift(v):
    """Wavelength factor sqrt((1 - v/c) / (1 + v/c)) for LOS velocity v (constants.py:31-45)."""
    beta = v / c
    return np.sqrt((1. - beta) / (1. + beta))


class Species:
    """An atom or ion: name ('NaI'), element ('Na'), ionisation stage string ('1'), mass [g]."""

    def __init__(self, name: str, element: str, ionizationState: str, mass: float) -> None:
        self.name = name
        self.element = element
        self.ionizationState = ionizationState
        self.mass = mass

    def __repr__(self):
        return "Species(%r)" % self.name


class SpeciesCollection:
    """A list of Species with lookup by name (constants.py:76-128)."""

    def __init__(self, speciesList: Optional[List[Species]] = None) -> None:
        self.speciesList: List[Species] = [] if speciesList is None else speciesList

    def findSpecies(self, nameSpecies: str) -> Optional[Species]:
        for sp in self.speciesList:
            if sp.name == nameSpecies:
                return sp
        print('Species', nameSpecies, 'was not found.')
        return None

    def listSpeciesNames(self) -> List[str]:
        return [sp.name for sp in self.speciesList]

    def addSpecies(self, species: Species) -> None:
        self.speciesList.append(species)


# (name, element, ionisation stage, mass in amu) -- constants.py:139-160
_SPECIES_TABLE = (
    ("NaI", "Na", "1", 22.99), ("KI", "K", "1", 39.0983), ("SiI", "Si", "1", 28.0855),
    ("SiII", "Si", "2", 28.0855), ("SiIII", "Si", "3", 28.0855), ("SiIV", "Si", "4", 28.0855),
    ("MgI", "Mg", "1", 24.305), ("MgII", "Mg", "2", 24.305), ("AlI", "Al", "1", 26.9815),
    ("CaI", "Ca", "1", 40.078), ("CaII", "Ca", "2", 40.078), ("TiI", "Ti", "1", 47.867),
    ("TiII", "Ti", "2", 47.867), ("CrI", "Cr", "1", 51.9961), ("MnI", "Mn", "1", 54.938),
    ("FeI", "Fe", "1", 55.845), ("CoI", "Co", "1", 58.933), ("NiI", "Ni", "1", 58.6934),
    ("OI", "O", "1", 15.999), ("CII", "C", "2", 12.011), ("SIII", "S", "3", 32.06),
    ("SIV", "S", "4", 32.06),
)


class AvailableSpecies(SpeciesCollection):
    """The species the NIST line list is filtered for."""

    def __init__(self) -> None:
        super().__init__([Species(n, el, ion, m * amu) for n, el, ion, m in _SPECIES_TABLE])
