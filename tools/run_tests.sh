#!/bin/bash
# GPU session: the -m gpu suite (optionally a -k selection) under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-t}
mkdir -p $OUT
K=${KSEL:+-k "$KSEL"}
timeout -k 10 ${TLIM:-900} python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -rA ${KSEL:+-k "$KSEL"} > $OUT/pytest.log 2>&1
rc=$?
tail -n 40 $OUT/pytest.log
exit $rc
