#!/bin/bash
# k_sigma_poly: segment kinds, truly isolated durations (one slot, no fork) of both parts and each alone,
# then PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-r03c}
mkdir -p $O
PROM_DEBUG=1 timeout -k 10 120 python -u bench.py --config C3 --no-cpu-baseline --no-projection --steps 20 --warmup 2 2>&1 | grep "\[prom\]" | head -3
for parts in 3 1 2; do
  (cd /tmp && PROM_SIG_PARTS=$parts PROM_PIPELINE=1 PROM_SIGMA_FORK=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/iso_p$parts -o run --output-format csv -- \
     python3 $GRAFT_REPO_ROOT/bench.py --config C3 --no-cpu-baseline --no-projection --steps 50 --warmup 5 > $O/iso_p$parts.log 2>&1) || { tail -20 $O/iso_p$parts.log; exit 1; }
  echo "parts $parts (PROM_PIPELINE=1, no fork):"; python3 tools/kstats.py $O/iso_p$parts/run_kernel_stats.csv 6
done
PROM_PIPELINE=1 PROM_SIGMA_FORK=0 TAG=${TAG:-r03c} KERN=k_sigma_poly bash tools/pmc_kernel.sh
exit 0
