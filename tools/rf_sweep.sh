#!/bin/bash
# Rows per front workgroup of k_sigma_tc (PROM_TC_RF) on C3 and C4x10: pipelined ms per step.
#   RFS="2 4 8" tools/rf_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/rf; mkdir -p $O
for rf in ${RFS:-2 4 8}; do
  for c in C3 C4x10; do
    PROM_TC_RF=$rf timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-projection --steps 300 --warmup 30 \
      > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('rf $rf', '$c', round(d['ms_per_step']*1e3,2), 'us step,', round(r['kernel_ms']*1e3,1), 'us', r['kernel'])"
  done
done
