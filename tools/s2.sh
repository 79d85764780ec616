# GPU session: the -m gpu suite, then 1-GPU benches of C2..C4 (no CPU baseline), each step time-limited.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
O=gpurun_out/${TAG:-s2}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -rA --timeout 300 --timeout-method thread ${KSEL:+-k "$KSEL"} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for c in ${CONFIGS:-C3 C2 C4}; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 50 --warmup 5 > $O/bench_$c.log 2>&1 || exit $?
  tail -1 $O/bench_$c.log | cut -c1-400
done
