#!/bin/bash
# Shard operators re-banded through hgm_mat_set_bands keep 4 lanes per band segment:
# per-rank SpMV times at N = 1..8 and the one-rank RCCL C4 solve.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/shard_order.py > gpurun_out/shard_order.log 2>&1 || exit $?
timeout -k 10 600 python -u scripts/shard_kernels.py > gpurun_out/shard_kernels.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --shard1 --no-cpu-baseline --steps 10 > gpurun_out/rccl1_bench.log 2>&1 || exit $?
