#!/bin/bash
# PMC passes (each its own rocprofv3 run, counters only -- no trace domains) over one tau-kernel
# variant.  Usage: tools/profile_pmc.sh <tag> [tune_tau args...]
#        PMC_SCRIPT=tools/rm_bench.py tools/profile_pmc.sh rm C2 --runs 1   (any python script + args)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${1:-tau}; shift
ARGS=${*:-"--variants 1 --exp 1 --reps 5"}
SCRIPT=${PMC_SCRIPT:-tools/tune_tau.py}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "== pass $i: $line"
  timeout -k 10 300 rocprofv3 --pmc $line --output-format csv -d $OUT/p$i -o p$i -- python3 $SCRIPT $ARGS > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; exit $rc; fi
done <<'PASSES'
GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64
SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SMEM SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FLOPS_FP64 SQ_WAIT_INST_LDS
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_LEVEL_WAVES SQ_INSTS_BRANCH
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
PASSES
find $OUT -name "*counter_collection.csv" | head
exit 0
