#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/shard_kernels.py 10 > gpurun_out/shard_kernels.log 2>&1 || exit $?
