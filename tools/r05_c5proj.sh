#!/bin/bash
# C5 full run against shard 0 of 8 on each axis (the strong-scaling projection's legs), env VARS per variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-r05c5}; mkdir -p $O
for v in ${VARS:-"X=0"}; do
  for leg in full phase wavelength; do
    a=""; [ $leg != full ] && a="--shard 0/8 --shard-axis $leg"
    f="$O/c5_${leg}_${v//\//_}.log"
    env ${v//,/ } timeout -k 10 300 python -u bench.py --config ${CFG:-C5} $a --no-cpu-baseline --no-projection --steps 30 --warmup 5 > "$f" 2>&1 || { tail -5 "$f"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1])
k=d['roofline'].get('kernels',{})
print('$v $leg', '%.4f ms' % d['ms_per_step'], {n: round(x.get('ms') or 0, 4) for n, x in k.items()})"
  done
done
