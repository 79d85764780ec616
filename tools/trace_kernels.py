#!/usr/bin/env python3
"""In-kernel timing of the transit pipeline (GPU box): builds libprom_hip_trace.so with -DPROM_TRACE,
runs one configuration and prints workgroup-0 step times of k_chords_w (wall clock, 10 ns ticks)
and per-wavefront cycle breakdowns of k_tau / k_columns8.

    python tools/trace_kernels.py [C2]
"""
import ctypes as C
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

from prometheus_amd import build  # noqa: E402

out = os.path.join(REPO, "prometheus_amd", "libprom_hip_trace.so")
srcs = [os.path.join(build.HERE, s) for s in build.SOURCES + build.HEADERS]
if not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(f) for f in srcs):
    build.build(force=True, extra=["-DPROM_TRACE"], out=out, objdir=os.path.join(build.HERE, "build_trace"))
os.environ["PROMETHEUS_AMD_LIB"] = out

from prometheus_amd import _native, configs, gasProperties, setupfile  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
cfg = configs.get(name)
if "H2O" in str(cfg["Species"]):
    gasProperties.register_molecular_table("H2O", configs.synthetic_molecular_table())
tr = setupfile.build_transit(cfg)
dev = _native.get_device(0)
host = tr._host_inputs()
dev.transit_set(tr._problem(dev, host, 0, len(tr.wavelength), 0.0))
lib = _native.load_library()
lib.prom_trace_read.restype = C.c_int32
lib.prom_trace_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int32, C.c_int32]
N = 1 << 20
buf = (C.c_ulonglong * N)()
for it in range(3):
    dev.transit_run()
    dev.synchronize()
    lib.prom_trace_read(buf, N, 1)
a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
n_orb = len(host["orb"])
print("k_order step times (us, workgroup of each phase, in time order; stamps 0 start, 7 loads issued+landed, "
      "1 classify+scan, 2 sort, 5 fetch+per-key work, 6 scans, 3 combine, 9 forward, 10 records, 4 tail+barrier, "
      "8 tables+end)")
for o in range(n_orb):
    t = a[o * 16: o * 16 + 11]
    if t[0] == 0:
        continue
    idx = sorted((i for i in range(11) if t[i] != 0), key=lambda i: t[i])   # stamps in time order
    d = ["%d->%d %5.2f" % (i, j, (t[j] - t[i]) * 0.01) for i, j in zip(idx, idx[1:])]
    print("  phase %2d: total %6.2f  steps %s" % (o, (t[8] - t[0]) * 0.01, " | ".join(d)))
kt = a[65536:600000 - (600000 - 65536) % 8].reshape(-1, 8)
kt = kt[kt[:, 7] > 0]
if len(kt):
    tot = kt[:, 6]
    win = kt[:, 5]
    print("k_tau_w per wave: records p50 %.0f p90 %.0f p99 %.0f max %.0f; lifetime ticks mean %.0f p50 %.0f p90 %.0f max %.0f"
          % (*np.percentile(win, [50, 90, 99, 100]), tot.mean(), *np.percentile(tot, [50, 90, 100])))
kc = a[600000:600000 + 2 * 100000].reshape(-1, 2)
kc = kc[kc[:, 1] > 0]
print("k_columns8 per wave lifetime ticks: mean %.0f p50 %.0f p90 %.0f (%d waves)"
      % (kc[:, 0].mean(), np.percentile(kc[:, 0], 50), np.percentile(kc[:, 0], 90), len(kc)))

# tau kernel wave timeline (wall clock, 10 ns ticks): start, end, HW_ID | XCC_ID << 32, record-lambda work
tl = a[700000:700000 + 4 * 80000].reshape(-1, 4)
tl = tl[tl[:, 1] > 0]
if len(tl):
    t0 = tl[:, 0].min()
    st = (tl[:, 0] - t0) * 0.01
    en = (tl[:, 1] - t0) * 0.01
    hw = tl[:, 2]
    heavy = (tl[:, 3] >> 62) & 1
    wk = tl[:, 3] & ((1 << 62) - 1)
    xcc = (hw >> 32) & 0xF
    print("tau kernel timeline (us): %d waves, span %.2f; starts p50 %.2f p90 %.2f max %.2f; ends p50 %.2f p90 %.2f p99 %.2f max %.2f"
          % (len(tl), en.max(), np.percentile(st, 50), np.percentile(st, 90), st.max(), *np.percentile(en, [50, 90, 99, 100])))
    dur = en - st
    print("  wave duration us: p10 %.2f p50 %.2f p90 %.2f max %.2f" % tuple(np.percentile(dur, [10, 50, 90, 100])))
    print("  record-lambda work per wave: p50 %.0f p90 %.0f p99 %.0f max %.0f, total %d" % (*np.percentile(wk, [50, 90, 99, 100]), wk.sum()))
    for t in np.arange(0, en.max() + 1, 1.0):
        print("  t=%5.1f us: %5d waves live, %5d started, %5d done" % (t, ((st <= t) & (en > t)).sum(), (st <= t).sum(), (en <= t).sum()))
    for x in range(8):
        m = xcc == x
        if m.any():
            print("  xcc %d: %5d waves, last end %.2f us, mean dur %.2f" % (x, m.sum(), en[m].max(), dur[m].mean()))
    for cls, m in (("heavy", heavy == 1), ("static", heavy == 0)):
        if m.any():
            busy = m & (wk > 0)
            print("  %s waves: %d (%d with work); duration p10 %.2f p50 %.2f p90 %.2f max %.2f; end p50 %.2f max %.2f; work p50 %.0f max %.0f"
                  % (cls, m.sum(), busy.sum(), *np.percentile(dur[m], [10, 50, 90, 100]), np.percentile(en[m], 50), en[m].max(),
                     np.percentile(wk[m], 50), wk[m].max()))
            if busy.any():
                for lo, hi in ((0, 8), (8, 16), (16, 32), (32, 64), (64, 1 << 30)):
                    mm = busy & (wk >= lo) & (wk < hi)
                    if mm.any():
                        print("    work [%d,%d): %5d waves, duration mean %.2f max %.2f" % (lo, hi, mm.sum(), dur[mm].mean(), dur[mm].max()))
    late = np.argsort(en)[-10:]
    print("  last-finishing waves (start, end, work):", [(round(float(st[i]), 2), round(float(en[i]), 2), int(wk[i])) for i in late])
