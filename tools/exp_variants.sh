# rocprofv3 kernel stats of C3 with experimental library variants (PROMETHEUS_AMD_LIB), pipeline serialised
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-expv}
mkdir -p $O
for v in ${VARIANTS}; do
  cd /tmp && PROMETHEUS_AMD_LIB=$GRAFT_REPO_ROOT/prometheus_amd/libprom_hip_$v.so PROM_PIPELINE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config ${CFG:-C3} --no-cpu-baseline --steps 20 --warmup 3 > $O/$v.log 2>&1 || exit $?
  echo "== $v"; grep -E "k_columns8|k_order|k_tau" $O/$v/run_kernel_stats.csv | python3 -c "
import sys,csv
for r in csv.reader(sys.stdin): print('%-40s avg %8.1f us' % (r[0][:40], float(r[3])/1e3))"
done
