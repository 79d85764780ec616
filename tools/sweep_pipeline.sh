# bench.py over pipeline depths / sigma-row fork settings: tools/sweep_pipeline.sh "C4 C3" "2 4 6 8" "0 1"
for c in ${1:-C4 C3 C2}; do for pl in ${2:-2 3 4}; do for f in ${3:-0 1}; do
PROM_PIPELINE=$pl PROM_SIGMA_FORK=$f timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/sw.log 2>&1 || exit 1
echo "$c pl=$pl fork=$f $(tail -1 gpurun_out/sw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(\"%.4e\" % d[\"value\"], \"%.4f\" % d[\"ms_per_step\"])")" | tee -a gpurun_out/sweep.txt
done; done; done
