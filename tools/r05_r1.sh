#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for r in 4 8; do PROM_TC_R1=$r TAG=r05h_r$r CFGS="${CFGS:-C4 C4x10}" bash tools/r05_quick.sh || exit 1; done
