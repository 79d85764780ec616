#!/bin/bash
# PMC passes over bench.py (one rocprofv3 run per pass, counters only), summarised for the kernels whose
# name contains each word of $KERN:  TAG=r03c KERN="k_sigma_poly k_order" CFG=C3 tools/pmc_kernel.sh
# (PASSES="line1;line2": only these counter sets)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-pmc}/pmc_${CFG:-C3}
mkdir -p $O
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  (cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc $line --output-format csv -d $O/p$i -o p$i -- \
     python3 $GRAFT_REPO_ROOT/bench.py --config ${CFG:-C3} --no-cpu-baseline --no-projection --steps 10 --warmup 2 > $O/p$i.log 2>&1) \
    || { echo "pass $i failed: $line"; tail -5 $O/p$i.log; exit 1; }
done <<PASSES
$(if [ -n "$PASSES" ]; then echo "$PASSES" | tr ';' '\n'; else cat <<'DEF'
GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU2
SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INSTS_BRANCH
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
DEF
fi)
PASSES
for k in ${KERN:-k_sigma}; do
  python3 tools/pmc_summary.py $O "$k" > $O/summary_$k.txt && echo "== $k" && cat $O/summary_$k.txt
done
exit 0
