#!/bin/bash
# Bench lines for the non-default workloads (BASELINE configs[2..4]); one JSON per run in
# gpurun_out/bench_<tag>.json.  RUNS: lines "tag | bench args".
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
RUNS=${RUNS:-"c3gcv_mgs | --workload c3gcv --steps 10 --warmup 2 --time-classes AB
c3gcv_cgs2 | --workload c3gcv --orth cgs2 --steps 10 --warmup 2 --time-classes AB
c3 | --workload c3 --steps 10 --warmup 2 --time-classes AB
c4 | --workload c4 --steps 5 --warmup 1 --time-classes AB
c5 | --workload c5 --steps 5 --warmup 1 --time-classes AB
c5m | --workload c5m --steps 5 --warmup 1 --time-classes AB"}
while IFS= read -r line; do
  [ -z "$line" ] && continue
  tag=$(echo "${line%%|*}" | xargs); args="${line#*|}"
  timeout -k 10 600 python bench.py $args --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 || { echo "FAIL $tag"; tail -20 gpurun_out/bench_$tag.log; exit 1; }
  grep '^{' gpurun_out/bench_$tag.log > gpurun_out/bench_$tag.json
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_$tag.json'))
print('$tag', d['value'], d['unit'], {k: round(v['avg_us'],1) for k,v in d.get('kernels',{}).items()}, d.get('gcv',''))"
done <<< "$RUNS"
