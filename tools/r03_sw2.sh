#!/bin/bash
# Variant libraries x configurations: pipelined bench line and the isolated per-kernel times (prom_transit_kernel_ms).
#   VARIANTS="base r4" CFGS="C3 C4x10" ENVS="PROM_SIG_PARTS=1" tools/r03_sw2.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-sw2}
mkdir -p $O
for c in ${CFGS:-C3}; do
for v in ${VARIANTS:-base}; do
for e in ${ENVS:-X=0}; do
  lib=prometheus_amd/libprom_hip_$v.so; [ "$v" = base ] && lib=prometheus_amd/libprom_hip.so
  f=$O/bench_${v}_${c}_${e//[^A-Za-z0-9]/_}.log
  env $e PROMETHEUS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-projection --steps 100 --warmup 10 ${BARGS} > $f 2>&1 || { tail -20 $f; exit 1; }
  echo "$v $c $e $(tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['roofline']['kernels']; print('%.4e' % d['value'], '%.4f ms' % d['ms_per_step'], 'single %.3f' % d['single_run_ms'], ' '.join('%s=%.1f' % (n, 1e3 * v['ms']) for n, v in k.items()))")"
done
done
done
exit 0
