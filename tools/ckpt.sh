#!/bin/bash
# Checkpoint on the committed tree: -m gpu suite, smoke, the default bench line (CPU legs +
# strong-scaling projection), rocprofv3 kernel stats pipelined and isolated (one slot, no fork), FETCH /
# WRITE traffic passes, the HBM microbenchmark.  Every GPU step has its own time limit; first failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T=${TAG:-ckpt}
O=$PWD/gpurun_out/$T
mkdir -p $O
has() { case " ${STEPS:-tests smoke bench stats traffic micro trace} " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
if has smoke; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log | cut -c1-200
fi
if has micro; then
  timeout -k 10 120 ./tools/microbench/hbm_peak > $O/hbm_peak.json || exit 1
  cat $O/hbm_peak.json
fi
for c in ${CFGS:-C3}; do
  if has bench; then
    extra=""; [ "$c" != C3 ] && extra="--no-cpu-baseline --no-projection"
    timeout -k 10 600 python -u bench.py --config $c $extra > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 1; }
    tail -1 $O/bench_$c.log > $O/bench_$c.json
    python3 -c "import json; d=json.load(open('$O/bench_$c.json')); print('$c', '%.4e' % d['value'], '%.4f ms' % d['ms_per_step'], d['roofline']['kernel'], '%.3f' % (d['roofline']['frac'] or 0))"
  fi
  if has stats; then
    for pipe in 4 1; do
      (cd /tmp && PROM_PIPELINE=$pipe PROM_SIGMA_FORK=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_${c}_p$pipe -o run --output-format csv -- \
         python3 $GRAFT_REPO_ROOT/bench.py --config $c --no-cpu-baseline --no-projection --steps 50 --warmup 5 > $O/stats_${c}_p$pipe.log 2>&1) \
        || { tail -20 $O/stats_${c}_p$pipe.log; exit 1; }
      echo "$c pipeline $pipe:"; python3 tools/kstats.py $O/stats_${c}_p$pipe/run_kernel_stats.csv 6
    done
  fi
  if has traffic; then
    mkdir -p $O/traffic_$c
    for k in FETCH_SIZE WRITE_SIZE; do
      (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $k --output-format csv -d $O/traffic_$c/$k -o $k -- \
         python3 $GRAFT_REPO_ROOT/bench.py --config $c --no-cpu-baseline --no-projection --steps 10 --warmup 2 > $O/traffic_$c/$k.log 2>&1) \
        || { echo "$k pass failed"; exit 1; }
    done
    python3 tools/traffic_summary.py $O/traffic_$c > $O/traffic_$c/summary.json
  fi
done
if has trace; then
  timeout -k 10 300 python -u tools/trace_kernels.py C3 > $O/trace_C3.txt 2>&1 || { tail -20 $O/trace_C3.txt; exit 1; }
  head -20 $O/trace_C3.txt
fi
exit 0
