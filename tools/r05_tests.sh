set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -rA --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -30; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
