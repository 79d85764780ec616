#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-r05e}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tcurve.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for p in 1 0; do
  PROM_TC_PERSIST=$p TAG=${TAG:-r05e}_p$p bash tools/r05_quick.sh || exit 1
done
