# pipeline depth x hardware queues per process (GPU_MAX_HW_QUEUES, default 4 on the box)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/hwq
for c in C3 C4; do for q in 4 8; do for d in 4 6 8; do
  GPU_MAX_HW_QUEUES=$q PROM_PIPELINE=$d timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/hwq/b_${c}_${q}_$d.log 2>&1 || exit 1
  echo "$c hwq=$q depth=$d $(tail -1 gpurun_out/hwq/b_${c}_${q}_$d.log | grep -o '"value": [0-9.e+]*' ) $(tail -1 gpurun_out/hwq/b_${c}_${q}_$d.log | grep -o '"ms_per_step": [0-9.]*')"
done; done; done
