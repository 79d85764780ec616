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
cmd = [build.hipcc()] + build.FLAGS + ["-DPROM_TRACE", "-o", out] + [os.path.join(build.HERE, s) for s in build.SOURCES]
subprocess.run(cmd, check=True, cwd=build.HERE)
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
print("k_order step times (us, workgroup of each phase): 1 load+scan | 2 sort | 3 fetch+scan | 4 records | "
      "5-7 - | 8 tables+end")
for o in range(n_orb):
    t = a[o * 16: o * 16 + 9]
    if t[0] == 0:
        continue
    d = np.diff(t) * 0.01
    print("  phase %2d: total %6.2f  steps %s" % (o, (t[8] - t[0]) * 0.01, " ".join("%5.2f" % v for v in d)))
kt = a[65536:600000 - (600000 - 65536) % 8].reshape(-1, 8)
kt = kt[kt[:, 7] > 0]
wall = (a[4000] - a[4002]) * 10.0  # ns, block 0 wave 0 lifetime
clk = a[4001] - a[4003]
print("clock64 ticks per ns (block 0 wave 0): %.3f" % (clk / max(wall, 1)))
pairs = kt[:, 4].sum()
print("k_tau_w per (wave, phase) mean ticks: sigma+windows %.0f, -, phases %.0f, -; records/phase %.1f; pairs %d"
      % tuple([kt[:, i].sum() / pairs for i in range(4) if i in (0, 2)] + [kt[:, 5].sum() / pairs, pairs]))
tot = kt[:, 6]
win = kt[:, 5]
print("window records per wave: p50 %.0f p90 %.0f p99 %.0f max %.0f" % tuple(np.percentile(win, [50, 90, 99, 100])))
for lo, hi in [(0, 4), (4, 16), (16, 64), (64, 256), (256, 10**9)]:
    m = (win >= lo) & (win < hi)
    if m.any():
        print("  window [%d,%d): %5d waves, lifetime mean %.0f max %.0f ticks" % (lo, hi, m.sum(), tot[m].mean(), tot[m].max()))
print("k_tau per wave lifetime ticks: mean %.0f  p10 %.0f  p50 %.0f  p90 %.0f  max %.0f  (%d waves)"
      % (tot.mean(), *np.percentile(tot, [10, 50, 90, 100]), len(tot)))
kc = a[600000:600000 + 2 * 100000].reshape(-1, 2)
kc = kc[kc[:, 1] > 0]
print("k_columns8 per wave lifetime ticks: mean %.0f p50 %.0f p90 %.0f (%d waves)"
      % (kc[:, 0].mean(), np.percentile(kc[:, 0], 50), np.percentile(kc[:, 0], 90), len(kc)))
