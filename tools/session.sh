#!/bin/bash
# One GPU session: the -m gpu suite, the default bench line (C3, CPU baseline legs), extra configs,
# rocprofv3 kernel stats of the default bench and FETCH_SIZE / WRITE_SIZE passes (separate runs, counters
# only).  Every GPU step has its own time limit and the steps are chained: the first failure ends the call.
#   TAG=r02b STEPS="tests bench extra stats traffic" CONFIGS="C2 C4" tools/session.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-s}
O=$PWD/gpurun_out/$TAG
mkdir -p $O
STEPS=${STEPS:-"tests bench extra stats traffic"}
CFG=${CFG:-C3}
has() { case " $STEPS " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -rA --timeout 300 --timeout-method thread ${KSEL:+-k "$KSEL"} > $O/pytest.log 2>&1 \
    || { tail -40 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
if has smoke; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log | cut -c1-300
fi
if has bench; then
  timeout -k 10 400 python -u bench.py --config $CFG > $O/bench_$CFG.log 2>&1 || { tail -20 $O/bench_$CFG.log; exit 1; }
  tail -1 $O/bench_$CFG.log | cut -c1-600
fi
if has extra; then
  for c in ${CONFIGS:-C2 C4}; do
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 100 --warmup 10 > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 1; }
    tail -1 $O/bench_$c.log | cut -c1-300
  done
fi
if has stats; then
  (cd /tmp && PROM_PIPELINE=${PIPE:-4} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_$CFG -o run --output-format csv -- \
     python3 $GRAFT_REPO_ROOT/bench.py --config $CFG --no-cpu-baseline --no-projection --steps 50 --warmup 5 > $O/stats_$CFG.log 2>&1) \
    || { tail -20 $O/stats_$CFG.log; exit 1; }
  python3 tools/kstats.py $O/stats_$CFG/run_kernel_stats.csv
fi
if has traffic; then
  mkdir -p $O/traffic_$CFG
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/traffic_$CFG/$c -o $c -- \
       python3 $GRAFT_REPO_ROOT/bench.py --config $CFG --no-cpu-baseline --no-projection --steps 10 --warmup 2 > $O/traffic_$CFG/$c.log 2>&1) \
      || { echo "$c pass failed"; exit 1; }
  done
  python3 tools/traffic_summary.py $O/traffic_$CFG > $O/traffic_$CFG/summary.json && grep -A6 "k_tau\|k_columns8\|k_order\|k_sig" $O/traffic_$CFG/summary.json | head -40
fi
exit 0
