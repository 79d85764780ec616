#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats CSV:  python tools/kstats.py <run_kernel_stats.csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 10]:
    print("%-44s %5s calls  avg %9.1f us  min %9.1f us  %5.1f%%" % (
        r["Name"].split("(")[0].replace("void ", "")[:44], r["Calls"], float(r["AverageNs"]) / 1e3,
        float(r["MinNs"]) / 1e3, float(r["Percentage"])))
