#!/usr/bin/env python3
"""D2H of R into a pooled pinned array vs ordinary memory (GPU box): median of 30 prom_transit_result calls.
    PROM_D2H_SPLIT=k python tools/d2h_probe.py C2"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from prometheus_amd import _native, configs, setupfile  # noqa: E402

tr = setupfile.build_transit(configs.get(sys.argv[1] if len(sys.argv) > 1 else "C2"))
dev = _native.get_device(0)
R = tr.sumOverChords(devices=[0])
pin = _native.host_array(R.shape)
plain = np.empty(R.shape)
plain[:] = 0
for name, out in (("pinned", pin), ("pageable", plain)):
    ts = []
    for _ in range(30):
        t = time.perf_counter()
        dev.transit_result(out=out)
        ts.append(time.perf_counter() - t)
    ms = float(np.median(ts)) * 1e3
    print("split=%s %-8s %.3f ms  %.1f GB/s" % (os.environ.get("PROM_D2H_SPLIT", "1"), name, ms,
                                                R.nbytes / ms / 1e6))
