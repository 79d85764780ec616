#!/bin/bash
# HBM traffic of the dominant kernel for the bench command: two rocprofv3 PMC passes (FETCH_SIZE,
# WRITE_SIZE; counters only), summarised into profiles-style JSON by tools/traffic_summary.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-r01}; shift
ARGS=${*:-"--steps 10 --warmup 2 --no-cpu-baseline"}
OUT=gpurun_out/traffic_$TAG
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o $c -- python3 bench.py $ARGS > $OUT/$c.log 2>&1
  rc=$?; echo "$c rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/$c.log; exit $rc; }
done
python3 tools/traffic_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
