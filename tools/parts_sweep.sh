#!/bin/bash
# k_tc_build part count sweep (PROM_TC_PARTS) on C3 and a C4x10 wavelength shard (1/8): ms per step and kernel ms.
#   PARTS="8 12 16" tools/parts_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/parts; mkdir -p $O
for p in ${PARTS:-8 12 16}; do
  for c in "C3" "C4x10 --shard 0/8 --shard-axis wavelength"; do
    PROM_TC_PARTS=$p timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-projection --steps 300 --warmup 30 \
      > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    tail -1 $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('parts $p', '$c', round(d['ms_per_step']*1e3,2), 'us', {k: round(v['kernel_ms']*1e3,2) for k, v in r.get('kernels', {}).items() if isinstance(v, dict) and v.get('kernel_ms')})"
  done
done
