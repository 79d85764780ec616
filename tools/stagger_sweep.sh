cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/stag
for c in C3 C4 C2; do for sv in 0 1; do
  PROM_SIG_STAGGER=$sv timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/stag/b_${c}_$sv.log 2>&1 || exit 1
  echo "$c stagger=$sv $(tail -1 gpurun_out/stag/b_${c}_$sv.log | cut -c1-200 | grep -o '"value": [0-9.e+]*, .*"ms_per_step": [0-9.]*')"
done; done
PROM_SIG_STAGGER=1 timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "pipelin or C3 or c3 or doppler or Doppler" > gpurun_out/stag/pytest.log 2>&1; tail -2 gpurun_out/stag/pytest.log

