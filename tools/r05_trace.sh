#!/bin/bash
# k_sigma_tc workgroup timelines (trace library) for CFGS, then the quick bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-r05f}; mkdir -p $O
for c in ${CFGS:-C3 C4x10}; do
  timeout -k 10 200 python -u tools/trace_sigma.py $c > $O/trace_$c.txt 2>&1 || { tail -5 $O/trace_$c.txt; exit 1; }
  cat $O/trace_$c.txt
done
bash tools/r05_quick.sh
