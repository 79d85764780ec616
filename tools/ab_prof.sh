#!/bin/bash
# rocprofv3 kernel-trace summaries of the bench with the planned tau path on and off (PROM_TAU_PLAN).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/ab
mkdir -p $OUT
for plan in 1 0; do
  PROM_TAU_PLAN=$plan timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/plan$plan -o run --output-format csv \
    -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/plan$plan.log 2>&1 || exit $?
  python3 - "$OUT/plan$plan" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-40s calls %4s avg %9.1f ns min %9s max %9s" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]), r["MinNs"], r["MaxNs"]))
PY
  grep -o '"value": [0-9.e+]*' $OUT/plan$plan.log
done
