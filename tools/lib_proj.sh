#!/bin/bash
# Default bench line (C3, with the C4x10 / C5 strong-scaling projection) per library variant:
#   tools/lib_proj.sh "base ilp8"      (prometheus_amd/libprom_hip_<v>.so; base = the default build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/lp
for v in $1; do
  lib=prometheus_amd/libprom_hip_$v.so; [ "$v" = base ] && lib=prometheus_amd/libprom_hip.so
  PROMETHEUS_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/lp/$v.log 2>&1 || { tail -20 gpurun_out/lp/$v.log; exit 1; }
  tail -1 gpurun_out/lp/$v.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); p = d['strong_scaling_projection']
print('$v', 'C3 %.4f ms' % d['ms_per_step'], ' '.join('%s full %.4f wl %.4f ph %.4f x%.2f' % (k, v['ms_full'], v['wavelength_shard']['ms_shard'], v['phase_shard']['ms_shard'], v['projected_speedup']) for k, v in p.items()))"
done
