"""Build libprom_hip.so in-tree for gfx950:  python -m prometheus_amd.build [-v]"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = ["csrc/prom_api.hip", "csrc/prom_transit.hip", "csrc/prom_fn.hip", "csrc/prom_mol.hip", "csrc/prom_tcurve.hip",
           "csrc/prom_rm.hip", "csrc/prom_sigma.hip", "csrc/prom_window.hip",
           "csrc/prom_tw.hip"]
HEADERS = ["csrc/prom_internal.h", "csrc/prom_device.h", "csrc/prom_tc.h", "csrc/faddeeva.h", "csrc/exp2_table.h",
           "csrc/exp2_table_body.h", "../include/prom_hip.h"]
OUT = os.path.join(HERE, "libprom_hip.so")
ARCH = os.environ.get("PROM_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=" + ARCH, "-ffp-contract=off", "-fPIC", "-Wall",
         "-Wno-unused-function"]
OBJDIR = os.path.join(HERE, "build")
# per-source flags (none at present; PROM_BUILD_NO_SRC_FLAGS drops them for A/B variant builds)
SRC_FLAGS = {}
if os.environ.get("PROM_BUILD_NO_SRC_FLAGS"):   # (variant builds, A/B of the per-source flags)
    SRC_FLAGS = {}


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(os.path.join(HERE, f)) <= t for f in SOURCES + HEADERS + ["build.py"])


def build(force: bool = False, verbose: bool = False, extra=(), out: str = OUT, objdir: str = OBJDIR,
          only=None) -> str:
    """One object per translation unit, compiled in parallel, then linked into the shared library
    (``extra``/``out``/``objdir``: variant builds such as the -DPROM_TRACE library of tools/trace_kernels.py;
    ``only``: compile just these sources with ``extra`` and link them with the default build's other objects)."""
    if not force and out == OUT and up_to_date() and not extra:
        return OUT
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(objdir, exist_ok=True)
    cc = hipcc()

    def compile_one(src: str) -> str:
        if only is not None and src not in only:
            return os.path.join(OBJDIR, os.path.basename(src).replace(".hip", ".o"))
        obj = os.path.join(objdir, os.path.basename(src).replace(".hip", ".o"))
        cmd = [cc] + FLAGS + SRC_FLAGS.get(src, []) + list(extra) + ["-c", os.path.join(HERE, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True, cwd=HERE)
        return obj

    with ThreadPoolExecutor(max_workers=min(len(SOURCES), os.cpu_count() or 1)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    cmd = [cc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-pthread", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True, cwd=HERE)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="-f" in sys.argv, verbose="-v" in sys.argv))
