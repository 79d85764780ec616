#!/bin/bash
# pipeline depth sweep (PROM_PIPELINE) on CFGS: bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for d in ${DEPTHS:-2 3 4 6 8}; do echo "== depth $d"; PROM_PIPELINE=$d TAG=r05v_d$d CFGS="${CFGS:-C3 C4x10}" bash tools/r05_quick.sh || exit 1; done
