cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/s1
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -rA --timeout 300 --timeout-method thread > gpurun_out/s1/pytest.log 2>&1 || exit $?
for c in C2 C3 C4 C5; do timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/s1/bench_$c.log 2>&1 || exit $?; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s1/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C3 --no-cpu-baseline --steps 50 --warmup 5 > $GRAFT_REPO_ROOT/gpurun_out/s1/prof.log 2>&1
