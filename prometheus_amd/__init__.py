"""prometheus_amd -- MI355X-native transit radiative-transfer core.

A drop-in for the per-(orbital phase, wavelength) optical-depth integrator of
CrazeXD/Prometheus (``Transit.sumOverChords``, pythonScripts/gasProperties.py:1160-1258):
the modules ``constants``, ``geometryHandler``, ``celestialBodies`` and ``gasProperties``
mirror the reference's ``pythonScripts`` package; the arithmetic runs in hand-written HIP
kernels for gfx950 behind the C-ABI of ``libprom_hip.so`` (include/prom_hip.h).
"""
__version__ = "0.1.0"

from . import constants, geometryHandler, celestialBodies  # noqa: F401  (pure host modules)


def native_available() -> bool:
    """True when libprom_hip.so loads and at least one GPU is visible."""
    from . import _native
    try:
        return _native.device_count() > 0
    except _native.NativeUnavailable:
        return False
