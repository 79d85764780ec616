#!/bin/bash
# Round-3 baseline on the committed tree: counter list, isolated (PROM_PIPELINE=1) kernel stats of C3,
# the pipelined C3 bench line without the CPU legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/${TAG:-r03a}
mkdir -p $O
if [ -n "$KSEL" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -rA --timeout 300 --timeout-method thread -k "$KSEL" > $O/pytest.log 2>&1 \
    || { tail -40 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
(cd /tmp && timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1); echo "list rc=$?"
grep -o "SQ_[A-Z0-9_]*" $O/counters.txt | sort -u > $O/sq_counters.txt || true
wc -l $O/sq_counters.txt
(cd /tmp && PROM_PIPELINE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/iso -o run --output-format csv -- \
   python3 $GRAFT_REPO_ROOT/bench.py --config C3 --no-cpu-baseline --steps 50 --warmup 5 > $O/iso.log 2>&1) \
  || { tail -20 $O/iso.log; exit 1; }
python3 tools/kstats.py $O/iso/run_kernel_stats.csv
timeout -k 10 300 python -u bench.py --config C3 --no-cpu-baseline > $O/bench_C3.log 2>&1 || { tail -20 $O/bench_C3.log; exit 1; }
tail -1 $O/bench_C3.log | cut -c1-400
exit 0
