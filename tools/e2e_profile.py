#!/usr/bin/env python3
"""Where the end-to-end time of one Transit.sumOverChords goes (GPU box): host inputs, problem marshalling,
prom_transit_set, prom_transit_run (+ sync), prom_transit_result (D2H of R), per stage, median of 20 calls.
    python tools/e2e_profile.py [C2]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from prometheus_amd import _native, configs, setupfile  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
tr = setupfile.build_transit(configs.get(name))
dev = _native.get_device(0)
for _ in range(3):
    tr.sumOverChords(devices=[0])
Rbuf = _native.host_array((len(tr.spatialGrid.constructOrbphaseAxis()), len(tr.wavelength)))
Rbuf[:] = 0.0
st = {k: [] for k in ("host_inputs", "problem", "set", "run_stats", "result_pinned", "total", "sumOverChords")}
for _ in range(20):
    t0 = time.perf_counter()
    host = tr._host_inputs()
    t1 = time.perf_counter()
    prob = tr._problem(dev, host, 0, len(tr.wavelength), 0.0)
    t2 = time.perf_counter()
    dev.transit_set(prob)
    t3 = time.perf_counter()
    dev.transit_run(stats=True)
    t4 = time.perf_counter()
    R = dev.transit_result(out=Rbuf)
    t5 = time.perf_counter()
    tr.sumOverChords(devices=[0])
    t6 = time.perf_counter()
    for k, v in zip(st, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t5 - t0, t6 - t5)):
        st[k].append(v * 1e3)
print(name, "R", R.shape, "%.1f MB" % (R.nbytes / 1e6), "(result: into a reused pinned array; sumOverChords: a new one from the pool)")
for k, v in st.items():
    print("  %-14s median %7.3f ms" % (k, float(np.median(v))))
