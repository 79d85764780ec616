#!/bin/bash
# quick GPU check: selected -m gpu tests (KSEL), then bench lines for CFGS (env passed through)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-r05q}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q -rA --timeout 120 --timeout-method thread ${KSEL:+-k "$KSEL"} > $O/pytest.log 2>&1 \
    || { grep -E "FAIL|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for c in ${CFGS:-C3 C4x10}; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-projection --steps 200 --warmup 20 > $O/bench_$c.log 2>&1 || { tail -5 $O/bench_$c.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$c.log').read().strip().splitlines()[-1])
k=d['roofline'].get('kernels',{})
print('$c', '%.4e' % d['value'], '%.4f ms' % d['ms_per_step'], 'single %.4f' % (d.get('single_run_ms') or 0), {n: round(v.get('ms') or 0, 4) for n, v in k.items()}, 'frac %.3f' % (d['roofline'].get('frac') or 0))"
done
