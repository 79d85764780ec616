#!/usr/bin/env python3
"""Per-launch FETCH_SIZE / WRITE_SIZE of each kernel from tools/bench_traffic.sh output (kB -> bytes).
gfx950 note (MI355X_MICROARCH.md, HBM): FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane)
coalesced stream; other access widths are uncalibrated.  hbm_bytes_per_launch applies that
correction (2 * FETCH_SIZE + WRITE_SIZE, kB -> bytes); the raw counter sum is kept beside it as
hbm_bytes_per_launch_raw."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
    per = collections.defaultdict(float)
    names = {}
    for row in csv.DictReader(open(f)):
        key = (row["Dispatch_Id"], row["Counter_Name"])
        per[key] += float(row["Counter_Value"])
        names[key] = row["Kernel_Name"]
    for (disp, cname), v in per.items():
        acc[names[(disp, cname)]][cname].append(v)
out = {}
for k, c in acc.items():
    short = k.split("(")[0].replace("void ", "")
    fetch = sum(c["FETCH_SIZE"]) / max(1, len(c["FETCH_SIZE"])) * 1024.0
    write = sum(c["WRITE_SIZE"]) / max(1, len(c["WRITE_SIZE"])) * 1024.0
    out[short] = {"launches": max(len(c["FETCH_SIZE"]), len(c["WRITE_SIZE"])), "fetch_bytes": fetch,
                  "write_bytes": write, "hbm_bytes_per_launch": 2 * fetch + write,
                  "hbm_bytes_per_launch_raw": fetch + write, "fetch_correction": 2.0}
json.dump(out, sys.stdout, indent=1)
