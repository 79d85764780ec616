#!/bin/bash
# A/B of k_sigma_tc rows per workgroup / rows per pass (PROM_TC_R, PROM_TC_NP) on C3 and C4x10: bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-r05d}; mkdir -p $O
for c in ${CFGS:-C3 C4x10}; do
  for v in ${VARIANTS:-"0 0" "8 4" "16 4" "16 8"}; do
    set -- $v
    PROM_TC_R=$1 PROM_TC_NP=$2 timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-projection --steps 200 --warmup 20 > $O/ab_${c}_$1_$2.log 2>&1 || { tail -5 $O/ab_${c}_$1_$2.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/ab_${c}_$1_$2.log').read().strip().splitlines()[-1])
k=d['roofline'].get('kernels',{})
print('$c R=$1 NP=$2', '%.4e' % d['value'], '%.4f ms' % d['ms_per_step'], {n: round(v.get('ms') or 0, 4) for n, v in k.items()})"
  done
done
