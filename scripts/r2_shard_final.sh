#!/bin/bash
# Dual strips limited to the full grid and 2-way shards: band/shard/RCCL tests and the per-rank
# shard costs at N = 1/2/4/8.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rccl.py -m gpu -x -q \
    -k "dual_strip or banded or paged_stream or shard or rccl" \
    --timeout 200 --timeout-method thread > gpurun_out/shard_final_tests.log 2>&1 || exit $?
echo "tests done"
timeout -k 10 900 python -u scripts/shard_kernels.py 10 > gpurun_out/shard_kernels.log 2>&1 || exit $?
