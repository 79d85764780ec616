#!/bin/bash
# Round-3 sigma-row session: Doppler parity tests, then bench + kernel stats per variant library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-r03b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -rA --timeout 300 --timeout-method thread ${KSEL:+-k "$KSEL"} > $O/pytest.log 2>&1 \
  || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
grep -h "poly rows" $O/pytest.log | head -20
for v in ${VARIANTS:-base}; do
  lib=prometheus_amd/libprom_hip_$v.so; [ "$v" = base ] && lib=prometheus_amd/libprom_hip.so
  for c in ${CONFIGS:-C3}; do
    PROMETHEUS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-projection --steps 200 --warmup 20 > $O/bench_${v}_$c.log 2>&1 || { tail -20 $O/bench_${v}_$c.log; exit 1; }
    echo "$v $c $(tail -1 $O/bench_${v}_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"%.4e\" % d[\"value\"], \"%.4f ms\" % d[\"ms_per_step\"], \"single %.3f ms\" % d[\"single_run_ms\"])")"
    for pipe in 4 1; do
      (cd /tmp && PROM_PIPELINE=$pipe PROMETHEUS_AMD_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/st_${v}_${c}_p$pipe -o run --output-format csv -- \
         python3 $GRAFT_REPO_ROOT/bench.py --config $c --no-cpu-baseline --no-projection --steps 50 --warmup 5 > $O/st_${v}_${c}_p$pipe.log 2>&1) || { tail -20 $O/st_${v}_${c}_p$pipe.log; exit 1; }
      echo "  pipeline $pipe:"; python3 tools/kstats.py $O/st_${v}_${c}_p$pipe/run_kernel_stats.csv 6
    done
  done
done
exit 0
