#!/usr/bin/env python3
"""Variant libraries of one translation unit (default: prom_sigma.hip) for GPU sweeps:
    python tools/build_variants.py NAME=-DMACRO=V[,-DMACRO2=W] ...
writes prometheus_amd/libprom_hip_NAME.so (select with PROMETHEUS_AMD_LIB, tools/variant_sweep.sh).  The
other objects come from the default build (python -m prometheus_amd.build)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from prometheus_amd import build as b  # noqa: E402

src = os.environ.get("VARIANT_SRC", "csrc/prom_sigma.hip")
for arg in sys.argv[1:]:
    name, flags = arg.split("=", 1)
    out = os.path.join(b.HERE, "libprom_hip_%s.so" % name)
    b.build(force=True, extra=tuple(flags.split(",")), out=out, objdir=os.path.join(b.HERE, "build_v_" + name),
            only=[src])
    print(out)
