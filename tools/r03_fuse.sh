#!/bin/bash
# Round-3 fused Doppler rows (k_sigma_poly TAU): -m gpu suite, bench lines with and without the fusion
# (PROM_SIG_TAU=0), rocprofv3 kernel stats of C3 pipelined and isolated.  First failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-r03f}
mkdir -p $O
has() { case " ${STEPS:-tests bench stats} " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -rA --timeout 300 --timeout-method thread ${KSEL:+-k "$KSEL"} > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; k=r['kernels']
print(sys.argv[2], '%.4e' % d['value'], '%.4f ms' % d['ms_per_step'], 'single %.3f' % d['single_run_ms'], ' '.join('%s=%.1f' % (n, (v.get('ms') or 0)*1e3) for n, v in k.items()))" $1 $2; }
if has bench; then
  for c in ${CFGS:-C3 C4 C4x10}; do
    for st in 1 0; do
      PROM_SIG_TAU=$st timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-projection --steps 100 --warmup 10 > $O/bench_${c}_t$st.log 2>&1 || { tail -20 $O/bench_${c}_t$st.log; exit 1; }
      tail -1 $O/bench_${c}_t$st.log > $O/bench_${c}_t$st.json
      summ $O/bench_${c}_t$st.json "$c tau=$st"
    done
  done
fi
if has stats; then
  for pipe in 4 1; do
    (cd /tmp && PROM_PIPELINE=$pipe timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats_C3_p$pipe -o run --output-format csv -- \
       python3 $GRAFT_REPO_ROOT/bench.py --config C3 --no-cpu-baseline --no-projection --steps 50 --warmup 5 > $O/stats_C3_p$pipe.log 2>&1) \
      || { tail -20 $O/stats_C3_p$pipe.log; exit 1; }
    echo "C3 pipeline $pipe:"; python3 tools/kstats.py $O/stats_C3_p$pipe/run_kernel_stats.csv 6
  done
fi
exit 0
