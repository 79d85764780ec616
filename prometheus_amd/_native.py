"""ctypes binding of libprom_hip.so (C-ABI declared in include/prom_hip.h).

The library is built in-tree for gfx950 (``python -m prometheus_amd.build`` or
``__graft_entry__.build()``).  There is no CPU fallback: if the library or a GPU is
missing, every compute call raises ``NativeUnavailable``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Dict, Optional, Sequence

import numpy as np

LIB_NAME = "libprom_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

PROM_OK = 0
STATUS = {-1: "PROM_E_ARG", -2: "PROM_E_HIP", -3: "PROM_E_NOMEM", -4: "PROM_E_STATE"}

DENSITY_BAROMETRIC = 1
DENSITY_HYDROSTATIC = 2
DENSITY_POWERLAW = 3
DENSITY_TORUS = 4
DENSITY_TABULATED = 5
DENSITY_GRIDDED = 6

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class NativeUnavailable(RuntimeError):
    """The HIP library is not built/loadable or no GPU is visible."""


class NativeError(RuntimeError):
    pass


class DensityModel(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32), ("p", C.c_double * 8)]


class Constituent(C.Structure):
    _fields_ = [("table_id", C.c_int32), ("is_molecule", C.c_int32), ("chi", C.c_double)]


class Scenario(C.Structure):
    _fields_ = [("density", DensityModel), ("body_x", _dp), ("body_y", _dp), ("shift", _dp),
                ("n_tabulated", _dp), ("T", C.c_double), ("n_constituents", C.c_int32),
                ("reserved", C.c_int32), ("constituents", C.POINTER(Constituent))]


class TransitProblem(C.Structure):
    _fields_ = [("n_wav", C.c_int64), ("wavelength", _dp), ("n_pr", C.c_int32), ("n_orb", C.c_int32),
                ("chord_y", _dp), ("chord_z", _dp), ("chord_fout", _dp), ("n_x", C.c_int32),
                ("n_scenarios", C.c_int32), ("x", _dp), ("delta_x", C.c_double), ("planet_y", _dp),
                ("planet_R", C.c_double), ("n_moons", C.c_int32), ("reserved", C.c_int32),
                ("moon_y", _dp), ("moon_R", _dp), ("scenarios", C.POINTER(Scenario)),
                ("cull_tau", C.c_double), ("options", C.c_int32), ("reserved2", C.c_int32),
                ("k_B", C.c_double), ("has_star", C.c_int32), ("star_table", C.c_int32),
                ("chord_rho", _dp), ("chord_clv", _dp), ("chord_star_shift", _dp)]


ABI_VERSION = 6
# prom_kernel_id order (prom_hip.h): the keys of Device.transit_kernel_ms
KERNEL_IDS = ("columns", "sigma", "order", "windows", "tau", "tc_build", "sigma_tc")
# prom_transit_stats.tau_kernel_variant // 10 -> the integration path the run took (prom_hip.h)
VARIANT_PATHS = {0: "k_tau (ocml exp, validation)", 1: "k_tau / k_tau_mol (table exp)", 2: "k_tau_w (windowed)",
                 3: "k_tau_p (planned windows)", 4: "k_tau_rm (stellar spectrum)",
                 8: "k_tc_build + k_sigma_tc (transmission curves)",
                 9: "k_tc_build + k_sigma_tw (transmission curves, target-window lookups)"}
OPT_OCML_EXP = 1
OPT_NO_MERGE = 2
OPT_NO_WINDOW = 4
OPT_DOPPLER_ROWS = 8


class TransitStats(C.Structure):
    _fields_ = [("ms_total", C.c_double), ("ms_density", C.c_double), ("ms_sigma", C.c_double),
                ("ms_tau", C.c_double), ("active_chords", C.c_int64), ("transparent_chords", C.c_int64),
                ("blocked_chords", C.c_int64), ("chord_lambda_evals", C.c_int64),
                ("tau_records", C.c_int64), ("exp_evals", C.c_int64),
                ("tau_kernel_variant", C.c_int32), ("exact_phases", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


# every exported symbol: name -> (restype, argtypes)
SIGNATURES = {
    "prom_abi_version": (C.c_int32, []),
    "prom_device_count": (C.c_int32, [_ip]),
    "prom_create": (C.c_int32, [C.c_int32, C.POINTER(C.c_void_p)]),
    "prom_destroy": (None, [C.c_void_p]),
    "prom_last_error": (C.c_char_p, [C.c_void_p]),
    "prom_synchronize": (C.c_int32, [C.c_void_p]),
    "prom_table_upload": (C.c_int32, [C.c_void_p, C.c_int64, _dp, _dp, C.c_double, _ip]),
    "prom_table_build_voigt": (C.c_int32, [C.c_void_p, C.c_int64, _dp, C.c_int32, _dp, _dp, _dp,
                                           C.c_double, C.c_double, C.c_double, _ip, _dp]),
    "prom_voigt_sigma": (C.c_int32, [C.c_void_p, C.c_int64, _dp, C.c_int32, _dp, _dp, _dp, C.c_double,
                                     C.c_double, _dp]),
    "prom_table_lookup": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int64, _dp, _dp]),
    "prom_table_free": (C.c_int32, [C.c_void_p, C.c_int32]),
    "prom_table_count": (C.c_int32, [C.c_void_p, _ip, _ip, C.POINTER(C.c_int64)]),
    "prom_molecular_free": (C.c_int32, [C.c_void_p, C.c_int32]),
    "prom_molecular_upload": (C.c_int32, [C.c_void_p, C.c_int32, _dp, C.c_int32, _dp, C.c_int64, _dp, _dp,
                                          C.c_double, _ip]),
    "prom_molecular_sigma": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int64, C.c_int32, _dp, C.c_double,
                                         C.c_int64, _dp, _dp]),
    "prom_number_density": (C.c_int32, [C.c_void_p, C.POINTER(DensityModel), C.c_int32, _dp, C.c_int64,
                                        _dp, _dp, _dp, _dp, _dp]),
    "prom_gridded_density": (C.c_int32, [C.c_void_p, C.c_int32, _dp, C.c_int32, _dp, C.c_int32, _dp, _dp,
                                         C.c_int64, _dp, _dp, _dp, _dp]),
    "prom_transit_set": (C.c_int32, [C.c_void_p, C.POINTER(TransitProblem)]),
    "prom_transit_run": (C.c_int32, [C.c_void_p, C.POINTER(TransitStats)]),
    "prom_transit_result": (C.c_int32, [C.c_void_p, _dp]),
    "prom_transit_columns": (C.c_int32, [C.c_void_p, _dp]),
    "prom_transit_band_stats": (C.c_int32, [C.c_void_p, C.c_int32, _dp, _dp, C.POINTER(C.c_int64), _dp]),
    "prom_transit_kernel_ms": (C.c_int32, [C.c_void_p, C.c_int32, _dp]),
    "prom_star_disk_flux": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int32, _dp, _dp, _dp, C.c_double, C.c_double,
                                        C.c_int64, _dp, _dp]),
    "prom_timing_begin": (C.c_int32, [C.c_void_p]),
    "prom_timing_end": (C.c_int32, [C.c_void_p, C.c_int32, _dp, _ip]),
    "prom_timing_stride": (C.c_int32, [C.c_void_p, C.c_int32]),
    "prom_host_alloc": (C.c_int32, [C.c_int64, C.POINTER(C.c_void_p)]),
    "prom_host_free": (C.c_int32, [C.c_void_p]),
}

_lib = None
_lib_lock = threading.Lock()


def load_library(path: Optional[str] = None):
    """Load (once) and type the C-ABI library.  Raises NativeUnavailable if absent."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or os.environ.get("PROMETHEUS_AMD_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise NativeUnavailable("%s not found: build it with `python -m prometheus_amd.build` "
                                    "(hipcc --offload-arch=gfx950); there is no CPU fallback" % p)
        try:
            lib = C.CDLL(p)
        except OSError as e:  # pragma: no cover - depends on the image
            raise NativeUnavailable("cannot load %s: %s" % (p, e))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.prom_abi_version() != ABI_VERSION:
            raise NativeUnavailable("ABI version mismatch")
        if path is None:
            _lib = lib
        return lib


def device_count() -> int:
    lib = load_library()
    n = C.c_int32(0)
    lib.prom_device_count(C.byref(n))
    return int(n.value)


class _PinnedBuffer:
    """A prom_host_alloc buffer exposed to numpy; returned to the pool when the last array over it dies."""

    def __init__(self, lib, ptr: int, shape):
        self._lib, self._ptr = lib, ptr
        self.__array_interface__ = {"shape": tuple(shape), "typestr": "<f8", "data": (ptr, False), "version": 3}

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self._lib.prom_host_free(C.c_void_p(self._ptr))
        except Exception:
            pass


def host_array(shape) -> Optional[np.ndarray]:
    """A float64 array of ``shape`` in page-locked memory from the library's pool (prom_host_alloc), or None
    when the pool's cap (PROM_PINNED_CAP_MB) is reached.  Device results copy into it with one DMA."""
    lib = load_library()
    n = int(np.prod(shape, dtype=np.int64)) * 8
    p = C.c_void_p()
    if lib.prom_host_alloc(n, C.byref(p)) != PROM_OK or not p.value:
        return None
    return np.asarray(_PinnedBuffer(lib, p.value, shape))


_pinned_usable: Optional[bool] = None


def pinned_copy(a) -> np.ndarray:
    """``a`` as a C-contiguous float64 array in the pinned pool (inputs re-sent on every call, such as the
    wavelength grid, then reach the device in one DMA), or an ordinary copy without a GPU or past the cap."""
    global _pinned_usable
    a = np.asarray(a, dtype=np.float64)
    if _pinned_usable is None:
        try:
            _pinned_usable = device_count() > 0
        except NativeUnavailable:
            _pinned_usable = False
    out = host_array(a.shape) if _pinned_usable and a.size else None
    if out is None:
        return np.array(a, dtype=np.float64, order="C")
    out[...] = a
    return out


def _d(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


class Device:
    """One prom_ctx (one GPU).  Not thread-safe; use one Device per host thread."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        n = device_count()
        if n == 0:
            raise NativeUnavailable("no HIP device visible (libprom_hip needs an MI355X / gfx950 GPU)")
        h = C.c_void_p()
        st = self.lib.prom_create(int(device), C.byref(h))
        if st != PROM_OK:
            raise NativeUnavailable("prom_create(%d) failed with %s" % (device, STATUS.get(st, st)))
        self.h = h
        self.device = int(device)
        self._keep = []
        # tables whose host objects were collected: freed at the next table or problem upload (a
        # finalizer may run while another thread is inside a call on this context)
        self._pending_free: list = []

    def close(self):
        if getattr(self, "h", None):
            self.lib.prom_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st: int, what: str):
        if st != PROM_OK:
            msg = self.lib.prom_last_error(self.h)
            raise NativeError("%s: %s (%s)" % (what, STATUS.get(st, st), msg.decode() if msg else ""))

    def synchronize(self):
        self._check(self.lib.prom_synchronize(self.h), "prom_synchronize")

    # ---- tables -----------------------------------------------------------------------
    def release_later(self, molecular: bool, table_id: int) -> None:
        """Queue a table for prom_table_free / prom_molecular_free (safe from finalizers)."""
        self._pending_free.append((bool(molecular), int(table_id)))

    def _drain_frees(self) -> None:
        while self._pending_free:
            mol, tid = self._pending_free.pop()
            self.table_free(tid, molecular=mol)

    def table_free(self, table_id: int, molecular: bool = False) -> None:
        fn = self.lib.prom_molecular_free if molecular else self.lib.prom_table_free
        self._check(fn(self.h, int(table_id)), "prom_molecular_free" if molecular else "prom_table_free")

    def table_count(self):
        """(live atomic tables, live molecular tables, device bytes they hold)."""
        a, m, b = C.c_int32(0), C.c_int32(0), C.c_int64(0)
        self._check(self.lib.prom_table_count(self.h, C.byref(a), C.byref(m), C.byref(b)), "prom_table_count")
        return int(a.value), int(m.value), int(b.value)

    def table_upload(self, x, y, offset: float) -> int:
        self._drain_frees()
        x, y = _f64(x), _f64(y)
        tid = C.c_int32(-1)
        self._check(self.lib.prom_table_upload(self.h, len(x), _d(x), _d(y), float(offset), C.byref(tid)),
                    "prom_table_upload")
        return int(tid.value)

    def table_build_voigt(self, x, line_w, line_g, line_coef, sigma_v, c_light, offset, want_host=True):
        self._drain_frees()
        x, lw, lg, lc = _f64(x), _f64(line_w), _f64(line_g), _f64(line_coef)
        out = np.empty_like(x) if want_host else None
        tid = C.c_int32(-1)
        self._check(self.lib.prom_table_build_voigt(self.h, len(x), _d(x), len(lw), _d(lw), _d(lg), _d(lc),
                                                    float(sigma_v), float(c_light), float(offset), C.byref(tid),
                                                    _d(out) if out is not None else None),
                    "prom_table_build_voigt")
        return int(tid.value), out

    def voigt_sigma(self, x, line_w, line_g, line_coef, sigma_v, c_light) -> np.ndarray:
        x, lw, lg, lc = _f64(x), _f64(line_w), _f64(line_g), _f64(line_coef)
        out = np.empty_like(x)
        self._check(self.lib.prom_voigt_sigma(self.h, x.size, _d(x), len(lw), _d(lw), _d(lg), _d(lc),
                                              float(sigma_v), float(c_light), _d(out)), "prom_voigt_sigma")
        return out

    def table_lookup(self, table_id: int, targets) -> np.ndarray:
        t = _f64(targets)
        out = np.empty_like(t)
        self._check(self.lib.prom_table_lookup(self.h, int(table_id), t.size, _d(t), _d(out)),
                    "prom_table_lookup")
        return out

    # ---- molecular ----------------------------------------------------------------------
    def molecular_upload(self, P, T, W, V, offset) -> int:
        self._drain_frees()
        P, T, W, V = _f64(P), _f64(T), _f64(W), _f64(V)
        assert V.shape == (len(P), len(T), len(W))
        tid = C.c_int32(-1)
        self._check(self.lib.prom_molecular_upload(self.h, len(P), _d(P), len(T), _d(T), len(W), _d(W), _d(V),
                                                   float(offset), C.byref(tid)), "prom_molecular_upload")
        return int(tid.value)

    def molecular_sigma(self, table_id, P, T, wav) -> np.ndarray:
        P, wav = _f64(P), _f64(wav)
        nc, nx = P.shape
        assert wav.shape[0] == nc
        nw = wav.shape[1]
        out = np.empty((nc, nx, nw))
        self._check(self.lib.prom_molecular_sigma(self.h, int(table_id), nc, nx, _d(P), float(T), nw, _d(wav),
                                                  _d(out)), "prom_molecular_sigma")
        return out

    # ---- density ------------------------------------------------------------------------
    def number_density(self, kind: int, params: Sequence[float], x, y, z, bx, by) -> np.ndarray:
        m = DensityModel()
        m.kind = int(kind)
        for i, v in enumerate(params):
            m.p[i] = float(v)
        x, y, z, bx, by = _f64(x), _f64(y), _f64(z), _f64(bx), _f64(by)
        out = np.empty((len(y), len(x)))
        self._check(self.lib.prom_number_density(self.h, C.byref(m), len(x), _d(x), len(y), _d(y), _d(z), _d(bx),
                                                 _d(by), _d(out)), "prom_number_density")
        return out

    def gridded_density(self, gx, gy, gz, values, px, py, pz) -> np.ndarray:
        """prom_gridded_density: scipy RegularGridInterpolator (linear) of values on (gx, gy, gz) at the
        points (px, py, pz); NaN outside the grid."""
        gx, gy, gz = _f64(gx), _f64(gy), _f64(gz)
        v = _f64(values)
        if v.shape != (len(gx), len(gy), len(gz)):
            raise ValueError("values must have shape (len(gx), len(gy), len(gz))")
        px, py, pz = np.broadcast_arrays(_f64(px), _f64(py), _f64(pz))
        px, py, pz = _f64(px), _f64(py), _f64(pz)
        out = np.empty(px.shape)
        self._check(self.lib.prom_gridded_density(self.h, len(gx), _d(gx), len(gy), _d(gy), len(gz), _d(gz), _d(v),
                                                  px.size, _d(px), _d(py), _d(pz), _d(out)), "prom_gridded_density")
        return out

    # ---- transit ------------------------------------------------------------------------
    def transit_set(self, prob: "TransitInputs"):
        self._drain_frees()
        self._keep = prob.keepalive
        self._check(self.lib.prom_transit_set(self.h, C.byref(prob.struct)), "prom_transit_set")
        self._shape = (prob.struct.n_orb, prob.struct.n_wav)
        self._n_atoms = prob.n_atoms
        self._n_pr = prob.struct.n_pr

    def transit_run(self, stats: bool = False):
        st = TransitStats() if stats else None
        self._check(self.lib.prom_transit_run(self.h, C.byref(st) if st is not None else None), "prom_transit_run")
        return st.as_dict() if st is not None else None

    def transit_result(self, out: Optional[np.ndarray] = None) -> np.ndarray:
        """R of the last run, [n_orb, n_wav]; ``out``: a C-contiguous float64 array of that shape to fill."""
        if out is None:
            out = np.empty(self._shape)
        elif out.shape != self._shape or out.dtype != np.float64 or not out.flags.c_contiguous:
            raise ValueError("transit_result: out must be a C-contiguous float64 array of shape %s" % (self._shape,))
        self._check(self.lib.prom_transit_result(self.h, _d(out)), "prom_transit_result")
        return out

    def timing_begin(self, stride: int = 1):
        """Start a timing window; events ride on every ``stride``-th run's tau dispatch."""
        self._check(self.lib.prom_timing_stride(self.h, int(stride)), "prom_timing_stride")
        self._check(self.lib.prom_timing_begin(self.h), "prom_timing_begin")

    def timing_end(self, max_runs: int = 4096) -> np.ndarray:
        """ms[run] = (NaN, NaN, tau_events, tau_device) of every timed run since timing_begin: the HIP
        event interval from the ordering kernel's completion to the tau kernel's, and the tau kernel's
        span on the device clock (first workgroup start -> last workgroup end; NaN unless k_tau_p)."""
        ms = np.zeros((max_runs, 4))
        n = C.c_int32(0)
        self._check(self.lib.prom_timing_end(self.h, max_runs, _d(ms), C.byref(n)), "prom_timing_end")
        return ms[:min(int(n.value), max_runs)]

    KERNEL_IDS = KERNEL_IDS

    def transit_kernel_ms(self, n_runs: int = 20) -> dict:
        """prom_transit_kernel_ms: mean device duration [ms] of each kernel of the current problem over
        n_runs serialized runs (one slot; dispatch-packet events), None for kernels the path does not launch."""
        ms = np.empty(len(self.KERNEL_IDS))
        self._check(self.lib.prom_transit_kernel_ms(self.h, int(n_runs), _d(ms)), "prom_transit_kernel_ms")
        return {k: (float(v) if np.isfinite(v) else None) for k, v in zip(self.KERNEL_IDS, ms)}

    def transit_columns(self) -> np.ndarray:
        out = np.empty((self._n_atoms, self._shape[0], self._n_pr))
        self._check(self.lib.prom_transit_columns(self.h, _d(out)), "prom_transit_columns")
        return out

    def transit_band_stats(self, bounds):
        """(sum, count, max) per phase of the last run's R over the band windows bounds[o][b] = (lo, hi)."""
        b = _f64(bounds)
        n_orb = self._shape[0]
        if b.ndim != 3 or b.shape[0] != n_orb or b.shape[2] != 2:
            raise ValueError("bounds must be [n_orb][n_bands][2]")
        s, c, m = np.empty(n_orb), np.empty(n_orb, dtype=np.int64), np.empty(n_orb)
        self._check(self.lib.prom_transit_band_stats(self.h, b.shape[1], _d(b), _d(s),
                                                     c.ctypes.data_as(C.POINTER(C.c_int64)), _d(m)),
                    "prom_transit_band_stats")
        return s, c, m


    # ---- stellar disk -----------------------------------------------------------------------
    def star_disk_flux(self, table_id: int, shift, clv, rho, dphi: float, drho: float, wavelength) -> np.ndarray:
        """prom_star_disk_flux: sum over disk cells (in order) of 10^interp(lambda / shift) clv dphi drho rho."""
        sh, cl, rh, w = _f64(shift), _f64(clv), _f64(rho), _f64(wavelength)
        if not (len(sh) == len(cl) == len(rh)):
            raise ValueError("shift, clv and rho need one value per disk cell")
        out = np.empty(w.shape)
        self._check(self.lib.prom_star_disk_flux(self.h, int(table_id), len(sh), _d(sh), _d(cl), _d(rh), float(dphi),
                                                 float(drho), w.size, _d(w), _d(out)), "prom_star_disk_flux")
        return out


class TransitInputs:
    """Owns the numpy arrays behind one prom_transit_problem (kept alive while in use)."""

    def __init__(self, *, wavelength, chord_y, chord_z, chord_fout, n_orb, x, delta_x, planet_y, planet_R,
                 moon_y, moon_R, scenarios, cull_tau=0.0, options=0, k_B=0.0, star=None):
        keep = []

        def arr(a):
            a = _f64(a)
            keep.append(a)
            return a

        s = TransitProblem()
        w = arr(wavelength)
        s.n_wav, s.wavelength = len(w), _d(w)
        cy, cz, cf = arr(chord_y), arr(chord_z), arr(chord_fout)
        s.n_pr, s.chord_y, s.chord_z, s.chord_fout = len(cy), _d(cy), _d(cz), _d(cf)
        s.n_orb = int(n_orb)
        xx = arr(x)
        s.n_x, s.x, s.delta_x = len(xx), _d(xx), float(delta_x)
        py = arr(planet_y)
        s.planet_y, s.planet_R = _d(py), float(planet_R)
        s.n_moons = len(moon_R)
        my, mr = arr(np.reshape(moon_y, (-1,)) if len(moon_R) else np.zeros(1)), arr(moon_R if len(moon_R) else np.zeros(1))
        s.moon_y, s.moon_R = _d(my), _d(mr)
        scs = (Scenario * len(scenarios))()
        n_atoms = 0
        for i, sc in enumerate(scenarios):
            d = scs[i]
            d.density.kind = int(sc["kind"])
            for j, v in enumerate(sc.get("params", ())):
                d.density.p[j] = float(v)
            if sc.get("body_x") is not None:
                d.body_x, d.body_y = _d(arr(sc["body_x"])), _d(arr(sc["body_y"]))
            d.shift = _d(arr(sc["shift"]))
            if sc.get("n_tabulated") is not None:
                d.n_tabulated = _d(arr(sc["n_tabulated"]))
            d.T = float(sc.get("T", 0.0))
            cons = sc["constituents"]
            ca = (Constituent * max(1, len(cons)))()
            for k, c in enumerate(cons):
                ca[k].table_id = int(c["table_id"])
                ca[k].is_molecule = int(bool(c.get("is_molecule", False)))
                ca[k].chi = float(c["chi"])
                n_atoms += 0 if c.get("is_molecule", False) else 1
            keep.append(ca)
            d.n_constituents = len(cons)
            d.constituents = ca
        keep.append(scs)
        s.n_scenarios = len(scenarios)
        s.scenarios = scs
        s.cull_tau = float(cull_tau)
        s.options = int(options)
        s.k_B = float(k_B)
        if star is not None:
            # {"table_id", "rho", "clv", "shift"}: stellar spectrum path (prom_hip.h has_star)
            s.has_star, s.star_table = 1, int(star["table_id"])
            s.chord_rho, s.chord_clv = _d(arr(star["rho"])), _d(arr(star["clv"]))
            s.chord_star_shift = _d(arr(star["shift"]))
        self.struct = s
        self.keepalive = keep
        self.n_atoms = n_atoms
        self.n_molecules = sum(1 for sc in scenarios for c in sc["constituents"] if c.get("is_molecule", False))


_default_device = int(os.environ.get("PROMETHEUS_DEVICE", "0"))


def set_default_device(device: int) -> None:
    """GPU used by calls that do not name one (table builds, plugin methods)."""
    global _default_device
    _default_device = int(device)


def default_device() -> int:
    return _default_device


_ctx_lock = threading.Lock()
_contexts: Dict[int, Device] = {}


def get_device(device: int = 0) -> Device:
    """Process-wide context of one GPU.  Serialise use with ``dev.lock`` (one host thread per
    device at a time; different devices run concurrently, ctypes drops the GIL)."""
    key = int(device)
    with _ctx_lock:
        d = _contexts.get(key)
        if d is None:
            d = Device(device)
            d.lock = threading.RLock()
            _contexts[key] = d
        return d
