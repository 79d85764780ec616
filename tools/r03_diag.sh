#!/bin/bash
# k_sigma_poly diagnostics: segment kinds, then PMC passes over each part alone (PROM_SIG_PARTS=1 / 2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-r03g}
mkdir -p $O
PROM_DEBUG=1 timeout -k 10 120 python -u bench.py --config C3 --no-cpu-baseline --no-projection --steps 20 --warmup 2 2>&1 | grep "\[prom\]" | head -3
for parts in 1 2; do
  i=0; mkdir -p $O/pmc_p$parts
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    (cd /tmp && PROM_SIG_PARTS=$parts PROM_PIPELINE=1 PROM_SIGMA_FORK=0 timeout -k 10 -s KILL 120 rocprofv3 --pmc $line --output-format csv -d $O/pmc_p$parts/p$i -o p$i -- \
       python3 $GRAFT_REPO_ROOT/bench.py --config C3 --no-cpu-baseline --no-projection --steps 10 --warmup 2 > $O/pmc_p$parts/p$i.log 2>&1) \
      || { echo "pass $i failed"; exit 1; }
  done <<'PASSES'
GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU
SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
PASSES
  echo "== parts $parts"; python3 tools/pmc_summary.py $O/pmc_p$parts k_sigma_poly | tee $O/pmc_p$parts/summary.txt
done
exit 0
