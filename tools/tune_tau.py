#!/usr/bin/env python3
"""A/B the fused tau kernel's variants on one GPU (tuning aid; not part of the product).

    python tools/tune_tau.py [--config C2] [--reps 20] [--variants 0,1,2] [--exp 1]
Prints per-variant mean k_tau time (live hipEvents) and checks R is identical across loop variants.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="0,1", help="1 = merge equal-column chords, 0 = no merge")
    ap.add_argument("--exp", default="1,0")
    a = ap.parse_args()
    from prometheus_amd import _native, configs, setupfile
    tr = setupfile.build_transit(configs.get(a.config))
    dev = _native.get_device(0)
    host = tr._host_inputs()
    out = {}
    Rref = None
    for e in [int(v) for v in a.exp.split(",")]:
        for lv in [int(v) for v in a.variants.split(",")]:
            opt = (0 if e else _native.OPT_OCML_EXP) | (0 if lv else _native.OPT_NO_MERGE)
            dev.transit_set(tr._problem(dev, host, 0, len(tr.wavelength), 0.0, opt))
            st = dev.transit_run(stats=True)
            for _ in range(3):
                dev.transit_run()
            dev.timing_begin()
            for _ in range(a.reps):
                dev.transit_run()
            ms = dev.timing_end(a.reps)
            R = dev.transit_result()
            if Rref is None:
                Rref = R
            key = "exp%d_merge%d" % (e, lv)
            out[key] = {"tau_ms": float(ms[:, 2].mean()), "tau_ms_min": float(ms[:, 2].min()),
                        "total_ms": float(ms[:, 3].mean()), "density_ms": float(ms[:, 0].mean()),
                        "variant": st["tau_kernel_variant"],
                        "max_rel_vs_first": float(np.max(np.abs(R / Rref - 1))),
                        "records": st["tau_records"], "active": st["active_chords"],
                        "exp_per_s": st["exp_evals"] / (ms[:, 2].mean() * 1e-3),
                        "cle_per_s": st["chord_lambda_evals"] / (ms[:, 2].mean() * 1e-3)}
            print(key, json.dumps(out[key]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
