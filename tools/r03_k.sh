#!/bin/bash
# Round-3 session: -m gpu suite, the C3 bench line (with the strong-scaling projection), sigma-kernel library
# variants on C3, C5 and C4 lines, rocprofv3 kernel stats of C3 (pipelined, isolated) and its FETCH / WRITE
# traffic.  Every GPU step has its own time limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-r03k}
mkdir -p $O
has() { case " ${STEPS:-tests bench variants extra stats traffic} " in *" $1 "*) return 0;; esac; return 1; }
summ() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; k=r['kernels']
print(sys.argv[2], '%.4e' % d['value'], '%.4f ms' % d['ms_per_step'], 'single %.3f' % d['single_run_ms'], ' '.join('%s=%.1f' % (n, (v.get('ms') or 0)*1e3) for n, v in k.items()))
for n, p in (d.get('strong_scaling_projection') or {}).items():
  print('  ', n, 'full %.4f' % p['ms_full'], 'wl %.4f %.2fx' % (p['wavelength_shard']['ms_shard'], p['wavelength_shard']['projected_speedup']), 'ph %.4f %.2fx' % (p['phase_shard']['ms_shard'], p['phase_shard']['projected_speedup']))" $1 $2; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -rA --timeout 300 --timeout-method thread ${KSEL:+-k "$KSEL"} > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
if has bench; then
  timeout -k 10 600 python -u bench.py --config C3 --no-cpu-baseline > $O/bench_C3.log 2>&1 || { tail -20 $O/bench_C3.log; exit 1; }
  tail -1 $O/bench_C3.log > $O/bench_C3.json; summ $O/bench_C3.json C3
fi
if has variants; then
  for v in ${VARIANTS:-m3 r4}; do
    PROMETHEUS_AMD_LIB=prometheus_amd/libprom_hip_$v.so timeout -k 10 300 python -u bench.py --config C3 --no-cpu-baseline --no-projection --steps 200 --warmup 20 > $O/bench_C3_$v.log 2>&1 || { tail -20 $O/bench_C3_$v.log; exit 1; }
    tail -1 $O/bench_C3_$v.log > $O/bench_C3_$v.json; summ $O/bench_C3_$v.json "C3 $v"
  done
fi
if has extra; then
  for c in ${CONFIGS:-C5 C4 C2}; do
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-projection --steps ${XSTEPS:-50} --warmup 5 > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 1; }
    tail -1 $O/bench_$c.log > $O/bench_$c.json; summ $O/bench_$c.json $c
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
if has traffic; then
  mkdir -p $O/traffic_C3
  for k in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -k 10 -s KILL 240 rocprofv3 --pmc $k --output-format csv -d $O/traffic_C3/$k -o $k -- \
       python3 $GRAFT_REPO_ROOT/bench.py --config C3 --no-cpu-baseline --no-projection --steps 10 --warmup 2 > $O/traffic_C3/$k.log 2>&1) \
      || { echo "$k pass failed"; exit 1; }
  done
  python3 tools/traffic_summary.py $O/traffic_C3 > $O/traffic_C3/summary.json
  python3 -c "
import json; d=json.load(open('$O/traffic_C3/summary.json'))
for k, v in d.items():
  if 'k_' in k: print(k, v['launches'], '%.2f MB' % (v['hbm_bytes_per_launch'] / 1e6))"
fi
exit 0
