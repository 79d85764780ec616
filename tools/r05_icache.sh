#!/bin/bash
# instruction-cache counters of k_sigma_tc on C3 (one rocprofv3 --pmc pass per set, counters only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-r05o}/pmc_${CFG:-C3}
mkdir -p $O
i=0
for line in "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU" "SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_REQ SQC_DCACHE_MISSES"; do
  i=$((i+1))
  (cd /tmp && timeout -k 5 -s KILL 90 rocprofv3 --pmc $line --output-format csv -d $O/p$i -o p$i -- \
     python3 $GRAFT_REPO_ROOT/bench.py --config ${CFG:-C3} --no-cpu-baseline --no-projection --steps 10 --warmup 2 > $O/p$i.log 2>&1) \
    || { echo "pass $i failed: $line"; tail -5 $O/p$i.log; }
done
python3 tools/pmc_summary.py $O k_sigma_tc
