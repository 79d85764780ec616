#!/usr/bin/env python3
"""Workgroup timeline of the sigma kernel (k_sigma_tc on the transmission-curve path, k_sigma_poly with
PROM_TCURVE=0; GPU box; libprom_hip_trace.so, every source built with -DPROM_TRACE): one run of a
configuration in isolation, then per part (front = oversize blocks, global records; main = LDS blocks) the
workgroups' start / end / duration percentiles on the wall clock (10 ns ticks).
    python tools/trace_sigma.py [C3]
"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

os.environ.setdefault("PROM_PIPELINE", "1")
os.environ.setdefault("PROM_SIGMA_FORK", "0")
os.environ["PROMETHEUS_AMD_LIB"] = os.path.join(REPO, "prometheus_amd", "libprom_hip_trace.so")
from prometheus_amd import _native, configs, setupfile  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
tr = setupfile.build_transit(configs.get(name))
dev = _native.get_device(0)
host = tr._host_inputs()
dev.transit_set(tr._problem(dev, host, 0, len(tr.wavelength), 0.0))
lib = _native.load_library()
rd = lib.prom_sig_trace_read if os.environ.get("PROM_TCURVE", "1") == "0" else lib.prom_tc_trace_read
rd.restype = C.c_int32
rd.argtypes = [C.POINTER(C.c_ulonglong), C.c_int32, C.c_int32]
N = 1 << 20
buf = (C.c_ulonglong * N)()
for it in range(3):
    rd(buf, N, 1)
    dev.transit_run()
    dev.synchronize()
rd(buf, N, 0)
# (k_sigma_tc's records: the first 2^19 entries; k_tc_build's stage stamps follow, tools/trace_tcb.py)
a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)[:1 << 19].reshape(-1, 4)
a = a[a[:, 1] > 0]
t0 = a[:, 0].min()
st, en = (a[:, 0] - t0) * 0.01, (a[:, 1] - t0) * 0.01
front = (a[:, 2] >> 33) & 1
lds = (a[:, 2] >> 32) & 1
print("%s sigma kernel: %d workgroups, span %.2f us" % (name, len(a), en.max()))
for nm, m in (("front (oversize, global records)", front == 1), ("main (LDS slices)", (front == 0) & (lds == 1))):
    if not m.any():
        continue
    d = en[m] - st[m]
    print("  %-34s n %5d  start p50 %6.2f p90 %6.2f max %6.2f | end p50 %6.2f p90 %6.2f max %6.2f | dur p10 %5.2f p50 %5.2f p90 %5.2f max %5.2f"
          % (nm, m.sum(), *np.percentile(st[m], [50, 90, 100]), *np.percentile(en[m], [50, 90, 100]),
             *np.percentile(d, [10, 50, 90, 100])))
# concurrency over time
ts = np.arange(0.0, en.max() + 1.0, 2.0)
conc = [int(((st <= t) & (en > t)).sum()) for t in ts]
print("  resident workgroups every 2 us:", " ".join(str(c) for c in conc))
# the slowest front workgroups' blocks
if (front == 1).any():
    idx = np.argsort(-(en - st) * (front == 1))[:10]
    print("  slowest front workgroups (block, row0, dur us, species kinds, largest slice):",
          ", ".join("(%d, %d, %.1f, %s, %d)" % (a[i, 2] & 0xffffffff, a[i, 3] & 0xffffffff, en[i] - st[i],
                                                 oct((a[i, 3] >> 32) & 0xfff), (a[i, 3] >> 44) & 0xffff) for i in idx))
    kz = np.array([any(((v >> (32 + 3 * s)) & 3) == 0 for s in range(4) if ((v >> 32) & 0xfff) >> (3 * s))
                   for v in a[:, 3]])
    kr = np.array([any(((v >> (32 + 3 * s)) & 3) == 3 for s in range(4) if ((v >> 32) & 0xfff) >> (3 * s))
                   for v in a[:, 3]])
    for nm, m in (("front, a species without guess", (front == 1) & kz), ("front, bucket directories", (front == 1) & kr & ~kz),
                  ("front, all guessed per block", (front == 1) & ~kz & ~kr)):
        if m.any():
            d = en[m] - st[m]
            print("  %-34s n %5d  dur p50 %5.2f p90 %5.2f max %5.2f" % (nm, m.sum(), *np.percentile(d, [50, 90, 100])))
