"""CPU-side checks of the C-ABI boundary: the library loads, exports every symbol declared in
include/prom_hip.h, and the product fails loudly (no CPU fallback) when no GPU is visible."""
import os
import re
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(REPO, "include", "prom_hip.h")).read()
    return sorted(set(re.findall(r"\b(prom_[a-z_]+)\s*\(", txt)))


def test_library_exports_header():
    from prometheus_amd import _native
    lib = _native.load_library()
    syms = header_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_native.SIGNATURES), set(syms) ^ set(_native.SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (prom_\w+)", out))
    assert set(syms) <= exported


def test_abi_version_and_no_device_here():
    from prometheus_amd import _native
    lib = _native.load_library()
    assert lib.prom_abi_version() == _native.ABI_VERSION == 6
    if _native.device_count() == 0:
        with pytest.raises(_native.NativeUnavailable):
            _native.Device(0)


def test_product_fails_loudly_without_gpu():
    from prometheus_amd import _native
    if _native.device_count() > 0:
        pytest.skip("a GPU is visible")
    from prometheus_amd import configs, setupfile
    with pytest.raises(_native.NativeUnavailable):
        setupfile.build_transit(configs.get("C1"))


def test_missing_library_is_an_error(tmp_path):
    from prometheus_amd import _native
    with pytest.raises(_native.NativeUnavailable):
        _native.load_library(str(tmp_path / "nope.so"))


def test_pinned_pool_argument_errors():
    """prom_host_alloc / prom_host_free reject bad arguments without touching a device."""
    import ctypes as C
    from prometheus_amd import _native
    lib = _native.load_library()
    p = C.c_void_p()
    E_ARG = -1
    assert _native.STATUS[E_ARG] == "PROM_E_ARG"
    assert lib.prom_host_alloc(-1, C.byref(p)) == E_ARG
    assert lib.prom_host_alloc(8, None) == E_ARG
    assert lib.prom_host_free(None) == E_ARG
    buf = np.zeros(4)
    assert lib.prom_host_free(C.c_void_p(buf.ctypes.data)) == E_ARG   # not a pool buffer


def test_header_documents_kernel_ids_and_variants():
    """prom_hip.h's prom_kernel_id enum is the binding's KERNEL_IDS (in order), every tens code of
    tau_kernel_variant the launcher can return is documented in the header, and the transmission-curve
    launcher times k_tc_build / k_sigma_tc under their own ids."""
    from prometheus_amd import _native
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "prom_hip.h")).read()
    enum = hdr[hdr.index("enum prom_kernel_id {"):]
    enum = enum[:enum.index("};")]
    ids = re.findall(r"PROM_K_(\w+) = (\d+)", enum)
    names = [n.lower() for n, v in ids if n != "COUNT"]
    assert [int(v) for n, v in ids] == list(range(len(ids)))
    assert tuple(names) == _native.KERNEL_IDS
    doc = hdr[hdr.index("int32_t tau_kernel_variant;"):hdr.index("tau_kernel_variant_exact_phases")]
    documented = {int(t) for t in re.findall(r"^\s+(\d)  \w", doc, re.M)}
    assert documented == set(_native.VARIANT_PATHS)
    src = "".join(open(os.path.join(root, "prometheus_amd", "csrc", f)).read()
                  for f in ("prom_transit.hip", "prom_mol.hip", "prom_tcurve.hip"))
    launched = {int(v) // 10 for v in re.findall(r"\*variant = (\d+)", src)}
    launched |= {int(v) // 10 for v in re.findall(r"\*variant = tw \? (\d+) \+ na : (?:\d+)", src)}
    launched |= {1, 2}   # *variant = na + (exp_mode ? (windowed ? 20 : 10) : 0)
    assert launched <= documented, launched - documented
    call = src[src.index("launch_tcurve(s, tr, rs"):]
    call = call[:call.index(";")]
    assert "PROM_K_SIGMA_TC" in call and "PROM_K_TC_BUILD" in call
