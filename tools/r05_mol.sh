#!/bin/bash
# molecular path: tests (molecular golden / KAT / C5 full-size), then C5 bench lines for each variant in VARS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-r05q}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multiscenario.py -q -x -k "C5 or molecular or mixed or three" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in ${VARS:-"X=0"}; do
  env ${v//,/ } timeout -k 10 300 python -u bench.py --config C5 --no-cpu-baseline --no-projection --steps 30 --warmup 5 > "$O/bench_C5_${v//\//_}.log" 2>&1 || { tail -5 "$O/bench_C5_${v//\//_}.log"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_C5_${v//\//_}.log').read().strip().splitlines()[-1])
k=d['roofline'].get('kernels',{})
print('$v', '%.4e' % d['value'], '%.4f ms' % d['ms_per_step'], {n: round(v.get('ms') or 0, 4) for n, v in k.items()}, 'frac %.3f' % (d['roofline'].get('frac') or 0))"
done
