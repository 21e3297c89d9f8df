#!/bin/bash
# A/B bench variants: each line of $VARIANTS is "ENV=.. ENV2=.. | extra bench args"; prints value + kernels.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
while IFS= read -r line; do
  [ -z "$line" ] && continue
  envs="${line%%|*}"; args="${line#*|}"
  timeout -k 10 300 env $envs python bench.py --workload ${WL:-c2} --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      $args > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/ab.log') if l.startswith('{')][-1])
print('[$line]', d['value'], {k: round(v['avg_us'],2) for k,v in d.get('kernels',{}).items()})"
  grep "host stats" gpurun_out/ab.log | tail -1
done <<< "$VARIANTS"
