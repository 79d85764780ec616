#!/bin/bash
# Round-5 counter session: PMC passes over k_sigma_tc (C3, C4x10) and k_tc_build, then C2 kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
T=${TAG:-r05c}
for c in ${CFGS:-C3 C4x10}; do
  TAG=$T CFG=$c KERN="k_sigma_tc k_tc_build k_columns8" bash tools/pmc_kernel.sh || exit 1
done
if [ -n "$C2STATS" ]; then
  TAG=$T STEPS="bench stats" CFGS=C2 bash tools/ckpt.sh || exit 1
fi
exit 0
