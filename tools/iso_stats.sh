#!/bin/bash
# Isolated kernel durations (PROM_PIPELINE=1: one run in flight, kernels do not share the CUs) of one
# config under rocprofv3 --kernel-trace --stats, once per environment variant given as arguments.
#   TAG=r02c CFG=C3 tools/iso_stats.sh "" "PROM_SIGMA_ROWS=0"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-iso}; CFG=${CFG:-C3}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
i=0
for v in "$@"; do
  i=$((i+1))
  echo "== variant $i: PROM_PIPELINE=1 $v"
  (cd /tmp && env PROM_PIPELINE=1 $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/iso$i -o run --output-format csv -- \
     python3 $GRAFT_REPO_ROOT/bench.py --config $CFG --no-cpu-baseline --steps 50 --warmup 5 > $O/iso$i.log 2>&1) \
    || { tail -20 $O/iso$i.log; exit 1; }
  tail -1 $O/iso$i.log | cut -c1-200
  python3 tools/kstats.py $O/iso$i/run_kernel_stats.csv
done
exit 0
