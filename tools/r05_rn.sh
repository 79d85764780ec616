#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for r in 8 4; do PROM_TC_RN=$r TAG=r05t_rn$r CFGS="${CFGS:-C3 C3}" bash tools/r05_quick.sh || exit 1; done
