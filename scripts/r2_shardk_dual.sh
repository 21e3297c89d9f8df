#!/bin/bash
# Per-rank A cost of the C4 shards under band_dual 0 / 1 / 2 (alternating order twice).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/shard_kernels.py 10 0,1,2,2,1,0 > gpurun_out/shard_kernels_dual.log 2>&1 || exit $?
