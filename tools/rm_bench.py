#!/usr/bin/env python3
"""Time the stellar-spectrum (CLV + Rossiter-McLaughlin) path on a named config against the flat star.

    python tools/rm_bench.py [C2] [--runs 5] [--vsini 5e6]

Prints one JSON line per mode with the single-run stage times of prom_transit_run (stats mode)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from prometheus_amd import _native, configs, setupfile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="C2")
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--vsini", type=float, default=5e6)
    ap.add_argument("--step", type=float, default=1e-10, help="stellar table spacing [cm]")
    a = ap.parse_args()
    cfg = configs.get(a.config)
    tr = setupfile.build_transit(cfg)
    tr.collect_stats = True
    g = cfg["Grids"]
    n_pts = None
    for mode in ("flat", "star"):
        if mode == "star":
            x, F = configs.synthetic_star_spectrum(g["lower_w"], g["upper_w"], step=a.step)
            hs = tr.planet.hostStar
            hs.addCLVparameters(0.34, 0.28)
            hs.addRMparameters(a.vsini, 0.4)
            hs.addFstarSpectrum(x, F)
        best = None
        for _ in range(a.runs):
            t0 = time.perf_counter()
            R = tr.sumOverChords(devices=[0])
            wall = time.perf_counter() - t0
            st = tr.last_stats[-1]
            if best is None or st["ms_total"] < best["ms_total"]:
                best = dict(st, wall_s=wall)
        n_pts = R.size
        print(json.dumps({"mode": mode, "config": a.config, "points": n_pts,
                          "pts_per_s_single_run": n_pts / (best["ms_total"] * 1e-3),
                          **{k: best[k] for k in ("ms_total", "ms_density", "ms_sigma", "ms_tau", "active_chords",
                                                  "transparent_chords", "blocked_chords", "tau_kernel_variant",
                                                  "wall_s")}}), flush=True)


if __name__ == "__main__":
    main()
