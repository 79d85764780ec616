#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel summary.
# Each GPU step has its own time limit; the script stops at the first fault/timeout/crash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/session.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/session.log
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"tests smoke bench prof"}
for s in $STEPS; do
  case $s in
    tests) step pytest_gpu 900 python -m pytest tests -q -m gpu -rA ;;
    rmtests) step pytest_rm 600 python -m pytest tests -q -m gpu -rA -k "stellar or native_loaded" -s ;;
    newtests) step pytest_new 600 python -m pytest tests -q -m gpu -rA -k "${KSEL:-native_loaded}" -s ;;
    rmbench) step rm_bench 600 python tools/rm_bench.py C2 --runs 3 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    benchfast) step bench 600 python bench.py --no-cpu-baseline ;;
    traffic) step traffic 700 bash tools/bench_traffic.sh ${TAG:-r01c} ;;
    trace) step trace 300 python tools/trace_kernels.py C2 ;;
    prof1) PROM_PIPELINE=1 step rocprof1 600 rocprofv3 --kernel-trace --stats -d $OUT/prof1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline ;;
  esac
done
exit 0
