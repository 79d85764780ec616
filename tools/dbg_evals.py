#!/usr/bin/env python3
"""Debug: R and exp-evaluation counts of one configuration under several environment settings (one process
per library): python tools/dbg_evals.py C3r "PROM_FUSED=0" "PROM_FUSED=1" "PROM_SIGMA_ROWS=0" ..."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

from prometheus_amd import configs, setupfile  # noqa: E402

name = sys.argv[1]
if name in ("C1", "C2", "C3", "C4", "C4x10", "C5"):
    cfg = configs.get(name)
else:
    cfg = json.loads(str(np.load(os.path.join(REPO, "tests", "golden", "transit_%s.npz" % name))["config"]))
tr = setupfile.build_transit(cfg)
tr.collect_stats = True
ref = None
for spec in sys.argv[2:]:
    for kv in spec.split(","):
        k, v = kv.split("=")
        os.environ[k] = v
    R = tr.sumOverChords(devices=[0])
    st = tr.last_stats[-1]
    if ref is None:
        ref = R
    d = np.max(np.abs(R - ref))
    print("%-40s variant %d exp_evals %d records %d  max|R - first| %.3e equal %s" % (
        spec, st["tau_kernel_variant"], st["exp_evals"], st["tau_records"], d, np.array_equal(R, ref)))
