#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
O=$PWD/gpurun_out/r03i
mkdir -p $O
timeout -k 10 120 ./tools/microbench/hbm_peak > $O/hbm_peak.json || exit 1
cat $O/hbm_peak.json
for sh in "" "--shard 0/8"; do
  f=$O/c4x10_$(echo "$sh" | tr -c 'a-z0-9' '_').log
  timeout -k 10 300 python -u bench.py --config C4x10 --no-cpu-baseline --no-projection --steps 100 --warmup 10 $sh > $f 2>&1 || { tail $f; exit 1; }
  tail -1 $f | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('C4x10 $sh ms/step %.4f' % d['ms_per_step'], {k: round(v['ms']*1e3,1) for k,v in r['kernels'].items() if v.get('ms')})"
done
TAG=r03i bash tools/r03_diag.sh > $O/diag.txt 2>&1 || { tail $O/diag.txt; exit 1; }
exit 0
