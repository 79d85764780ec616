#!/bin/bash
# Variant libraries: pipelined C3 bench line + isolated (one slot, no fork) kernel durations.
#   VARIANTS="base r4 m1r8" CFG=C3 tools/r03_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-sweep}
mkdir -p $O
for c in ${CFGS:-C3}; do
for v in ${VARIANTS:-base}; do
  lib=prometheus_amd/libprom_hip_$v.so; [ "$v" = base ] && lib=prometheus_amd/libprom_hip.so
  PROMETHEUS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-projection --steps 200 --warmup 20 > $O/bench_${v}_$c.log 2>&1 || { tail -20 $O/bench_${v}_$c.log; exit 1; }
  echo "$v $c $(tail -1 $O/bench_${v}_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"%.4e\" % d[\"value\"], \"%.4f ms\" % d[\"ms_per_step\"], \"single %.3f ms\" % d[\"single_run_ms\"])")"
  (cd /tmp && env ${ENVX} PROM_PIPELINE=1 PROM_SIGMA_FORK=0 PROMETHEUS_AMD_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/iso_${v}_$c -o run --output-format csv -- \
     python3 $GRAFT_REPO_ROOT/bench.py --config $c --no-cpu-baseline --no-projection --steps 50 --warmup 5 > $O/iso_${v}_$c.log 2>&1) || { tail -20 $O/iso_${v}_$c.log; exit 1; }
  python3 tools/kstats.py $O/iso_${v}_$c/run_kernel_stats.csv 5 | sed 's/^/    /'
done
done
exit 0
