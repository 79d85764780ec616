#!/usr/bin/env python3
"""Average per-dispatch PMC values per kernel from rocprofv3 counter_collection CSVs.
   python tools/pmc_summary.py gpurun_out/pmc_<tag> [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "k_tau"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        if sub not in row["Kernel_Name"]:
            continue
        key = (os.path.basename(f), row["Dispatch_Id"])
        agg[row["Counter_Name"]][key] += float(row["Counter_Value"])
        dur[row["Counter_Name"]].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
out = {}
for c, v in sorted(agg.items()):
    vals = list(v.values())
    out[c] = sum(vals) / len(vals)
    print("%-28s %14.5g   (n=%d, mean dur %.1f us)" % (c, out[c], len(vals), sum(dur[c]) / len(dur[c]) / 1e3))
