#!/bin/bash
# Alternating A/B comparison of two bench argument sets (noise control):
#   ARGS_X="..." ARGS_Y="..." WL=c2 REPS=3 bash scripts/ab_compare.sh
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in $(seq ${REPS:-3}); do
  for tag in X Y; do
    v="ARGS_$tag"; envv="ENV_$tag"
    env ${!envv} timeout -k 10 300 python bench.py --workload ${WL:-c2} --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline ${!v} > gpurun_out/ab.log 2>&1 || exit 1
    echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/ab.log | head -1) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/ab.log)"
  done
done
