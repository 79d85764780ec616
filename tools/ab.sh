#!/bin/bash
# A/B session: optional GPU tests (TESTS, KSEL), then per config (CFGS) and per environment variant (arguments):
# the pipelined bench line and the isolated kernel stats (PROM_PIPELINE=1 under rocprofv3 --kernel-trace --stats).
#   TAG=r06b CFGS="C3 C4x10" TESTS=tests/test_gpu_tcurve.py tools/ab.sh "" "PROM_TC_RG=1"
R=$(cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && pwd) || exit 2
cd "$R" || exit 2
export TMPDIR=/tmp
O=$R/gpurun_out/${TAG:-ab}; mkdir -p "$O"
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q -m gpu -rA --timeout 300 --timeout-method thread ${KSEL:+-k "$KSEL"} > "$O/pytest.log" 2>&1 \
    || { grep -E "FAIL|Error" "$O/pytest.log" | head -20; tail -30 "$O/pytest.log"; exit 1; }
  tail -1 "$O/pytest.log"
fi
[ $# -eq 0 ] && set -- ""
for c in ${CFGS:-C3}; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-projection --steps ${STEPS:-200} --warmup 20 > "$O/bench_${c}_$i.log" 2>&1 \
      || { tail -5 "$O/bench_${c}_$i.log"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/bench_${c}_$i.log').read().strip().splitlines()[-1])
k=d['roofline'].get('kernels',{})
print('$c [$v]', '%.4e' % d['value'], '%.4f ms' % d['ms_per_step'], {n: round(x.get('ms') or 0, 4) for n, x in k.items()}, 'frac %.3f' % (d['roofline'].get('frac') or 0))"
    if [ -z "$NOSTATS" ]; then
      (cd /tmp && env PROM_PIPELINE=1 $v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/iso_${c}_$i" -o run --output-format csv -- \
         python3 "$R/bench.py" --config $c --no-cpu-baseline --no-projection --steps 50 --warmup 5 > "$O/iso_${c}_$i.log" 2>&1) \
        || { tail -20 "$O/iso_${c}_$i.log"; exit 1; }
      python3 tools/kstats.py "$O/iso_${c}_$i/run_kernel_stats.csv" | head -${KTOP:-4}
    fi
  done
done
exit 0
