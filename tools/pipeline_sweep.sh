#!/bin/bash
# Throughput vs run-pipeline depth (PROM_PIPELINE slots/streams) and HIP hardware queues.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for q in 4 8; do
  for d in 2 4 6 8; do
    v=$(GPU_MAX_HW_QUEUES=$q PROM_PIPELINE=$d timeout -k 10 120 python bench.py --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.e+]*\|"tau_ms": [0-9.e+-]*' | tr '\n' ' ')
    echo "queues $q depth $d: $v"
  done
done
