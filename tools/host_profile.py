#!/usr/bin/env python3
"""cProfile of the host side of one sumOverChords (GPU box: the tables are built on the device):
200 x (Transit._host_inputs + Transit._problem), top functions by cumulative time.
    python tools/host_profile.py [C2]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from prometheus_amd import _native, configs, setupfile  # noqa: E402

tr = setupfile.build_transit(configs.get(sys.argv[1] if len(sys.argv) > 1 else "C2"))
dev = _native.get_device(0)
tr.sumOverChords(devices=[0])


def work():
    for _ in range(200):
        host = tr._host_inputs()
        tr._problem(dev, host, 0, len(tr.wavelength), 0.0)


pr = cProfile.Profile()
pr.enable()
work()
pr.disable()
pstats.Stats(pr).sort_stats("cumulative").print_stats(25)
