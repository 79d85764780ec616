"""Debug: C2 single-device repeatability, shards, and against the windowed path."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from prometheus_amd import configs, setupfile  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
tr = setupfile.build_transit(configs.get(name))
R1 = tr.sumOverChords(devices=[0])
R2 = tr.sumOverChords(devices=[0])
R3 = tr.sumOverChords(devices=[0, 0])
os.environ["PROM_TCURVE"] = "0"
R0 = tr.sumOverChords(devices=[0])
for nm, X in (("repeat", R2), ("2 shards", R3), ("windowed path", R0)):
    d = np.abs(X - R1).max(axis=1)
    print(nm, "max |dR| per row:", " ".join("%.2e" % v for v in d))
