#!/usr/bin/env python3
"""Stage timeline of k_tc_build (GPU box; libprom_hip_trace.so built with -DPROM_TRACE): one run of a
configuration on the transmission-curve path in isolation, then per stage (phase sums, node sums, hand-off,
last-arriver coefficients) the workgroups' duration percentiles and the kernel's span, on the wall clock
(10 ns ticks).
    python tools/trace_tcb.py [C3]
"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

os.environ.setdefault("PROM_PIPELINE", "1")
os.environ["PROMETHEUS_AMD_LIB"] = os.path.join(REPO, "prometheus_amd", "libprom_hip_trace.so")
from prometheus_amd import _native, configs, setupfile  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
tr = setupfile.build_transit(configs.get(name))
dev = _native.get_device(0)
host = tr._host_inputs()
dev.transit_set(tr._problem(dev, host, 0, len(tr.wavelength), 0.0))
lib = _native.load_library()
rd = lib.prom_tc_trace_read
rd.restype = C.c_int32
rd.argtypes = [C.POINTER(C.c_ulonglong), C.c_int32, C.c_int32]
N = 1 << 20
buf = (C.c_ulonglong * N)()
for it in range(3):
    rd(buf, N, 1)
    dev.transit_run()
    dev.synchronize()
rd(buf, N, 0)
a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)[1 << 19:].reshape(-1, 8)
a = a[a[:, 0] > 0]
t0 = a[:, 0].min()
t = (a[:, :5] - t0) * 0.01
last = (a[:, 6] >> 16) & 1
L = a[:, 6] & 0xffff
ch = a[:, 5] & 0xff
print("%s k_tc_build: %d workgroups, span %.2f us, last arrivers %d, chains with work %d" %
      (name, len(a), t[:, 4].max(), last.sum(), int((ch * 4 < np.maximum(L, 1)).sum())))
sw = np.where(a[:, 7] > 0, (a[:, 7] - t0) * 0.01, np.nan)   # (early-exit chains stamp no sweep end)
for nm, d in (("start", t[:, 0]), ("sweep (loads)", sw - t[:, 0]), ("reductions", t[:, 1] - sw),
              ("phase sums", t[:, 1] - t[:, 0]), ("node sums", t[:, 2] - t[:, 1]),
              ("hand-off", t[:, 3] - t[:, 2]), ("coefficients (last)", (t[:, 4] - t[:, 3])[last == 1]),
              ("end", t[:, 4])):
    d = d[np.isfinite(d)]
    if len(d):
        print("  %-22s p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f" % (nm, *np.percentile(d, [10, 50, 90, 100])))
print("  L per phase:", " ".join(str(int(x)) for x in np.unique(L)))
