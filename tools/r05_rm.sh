#!/bin/bash
# stellar-spectrum path: tests, then the C2 rotating-star run for each variant in VARS ("ENV=V ...")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/${TAG:-r05m}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_star_methods.py -q -x -k "stellar or star or rm" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in ${VARS:-"X=0"}; do
  env ${v//,/ } timeout -k 10 300 python -u tools/rm_bench.py C2 --runs 5 > $O/rm_$v.txt 2>&1 || { tail -5 $O/rm_$v.txt; exit 1; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$O/rm_$v.txt') if l.startswith('{')][-1]
print('$v', 'star ms_tau %.3f ms_total %.3f' % (d['ms_tau'], d['ms_total']))"
done
