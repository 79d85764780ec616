"""Transmission-curve diagnostics: per-phase active chords and table octaves (PROM_DEBUG), exp counts."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("PROM_DEBUG", "1")
from prometheus_amd import configs, setupfile  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
tr = setupfile.build_transit(configs.get(name))
tr.collect_stats = True
R = tr.sumOverChords(devices=[0])
print(name, tr.last_stats[-1])
