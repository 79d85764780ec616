# bench.py + rocprofv3 kernel stats per library variant (prometheus_amd/libprom_hip_<v>.so; "base" = the
# default build): tools/variant_sweep.sh "base s1024f1" "C3 C4"
export TMPDIR=/tmp
for v in $1; do for c in ${2:-C3}; do
  lib=prometheus_amd/libprom_hip_$v.so; [ "$v" = base ] && lib=prometheus_amd/libprom_hip.so
  PROMETHEUS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/vs.log 2>&1 || exit 1
  echo "$v $c $(tail -1 gpurun_out/vs.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"%.4e\" % d[\"value\"], \"%.4f\" % d[\"ms_per_step\"])")" | tee -a gpurun_out/variants.txt
  PROMETHEUS_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/vs_${v}_${c} -o run --output-format csv -- python3 -u bench.py --config $c --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/vs_prof.log 2>&1 || exit 1
  f=$(find gpurun_out/vs_${v}_${c} -name "run_kernel_stats.csv" | head -1)
  python3 - "$f" "$v $c" <<'PY' | tee -a gpurun_out/variants.txt
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "sigma_rows" in r["Name"] or "k_tau_p" in r["Name"]:
        print("   ", sys.argv[2], r["Name"][:40], "avg %.1f us" % (float(r["AverageNs"]) / 1e3), "calls", r["Calls"])
PY
  rm -rf gpurun_out/vs_${v}_${c}
done; done
