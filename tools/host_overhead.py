#!/usr/bin/env python3
"""Host cost of prom_transit_run (GPU box): enqueue time per run vs GPU time per run, with and
without the bench's stage events."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402,F401

from prometheus_amd import _native, configs, setupfile  # noqa: E402

tr = setupfile.build_transit(configs.get(sys.argv[1] if len(sys.argv) > 1 else "C2"))
dev = _native.get_device(0)
host = tr._host_inputs()
# optional second argument k: only the first 1/k of the wavelengths (one rank's shard of a k-way split)
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
n_w = (len(tr.wavelength) // k + 255) // 256 * 256 if k > 1 else len(tr.wavelength)
dev.transit_set(tr._problem(dev, host, 0, n_w, 0.0))
for _ in range(5):
    dev.transit_run()
dev.synchronize()
N = 200
print("PROM_PIPELINE", os.environ.get("PROM_PIPELINE", "2"))
for timing in (False, True):
    if timing:
        dev.timing_begin()
    t0 = time.perf_counter()
    for _ in range(N):
        dev.transit_run()
    t1 = time.perf_counter()
    dev.synchronize()
    t2 = time.perf_counter()
    if timing:
        ms = dev.timing_end(max_runs=N)
    print("timing=%s: enqueue %.1f us/run, total %.1f us/run" % (timing, (t1 - t0) / N * 1e6, (t2 - t0) / N * 1e6))
t0 = time.perf_counter()
for _ in range(N):
    dev.lib.prom_abi_version()
t1 = time.perf_counter()
print("bare ctypes call %.2f us" % ((t1 - t0) / N * 1e6))
