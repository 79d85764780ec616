# rocprofv3 kernel stats of one bench config with the pipeline serialised (PROM_PIPELINE=1): per-kernel
# durations without overlap between the four run slots.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-prof}
mkdir -p $O
for c in ${CONFIGS:-C3}; do
  cd /tmp && PROM_PIPELINE=${PIPE:-1} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --no-cpu-baseline --steps 30 --warmup 5 > $O/$c.log 2>&1 || exit $?
  python3 - $O/$c/run_kernel_stats.csv <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print("%-60s %6s calls avg %9.1f us  min %9.1f us  %5.1f%%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])/1e3, float(r["MinNs"])/1e3, float(r["Percentage"])))
PY
done
