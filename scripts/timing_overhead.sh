#!/bin/bash
# C2 bench under timing / sync-event variants (noise check: each variant twice).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for rep in 1 2; do
for v in 0 1; do
  HGM_SYNC_EVENT_NOFENCE=$v timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/t.log 2>&1 || exit 1
  echo "nofence=$v $(grep -o '"value": [0-9.]*' gpurun_out/t.log | head -1) $(grep -o '"residual_norm_last": [0-9.e-]*' gpurun_out/t.log)"
done
done
