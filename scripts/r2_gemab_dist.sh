#!/bin/bash
# m-space Gram error monitor on the sharded path: 2-rank emulation, one-rank RCCL, and the C4
# solve on a one-rank communicator.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rccl.py -x -v --timeout 300 \
    --timeout-method thread -k "shard or rccl or ab_gram" > gpurun_out/gemab_dist_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --shard1 --no-cpu-baseline --steps 10 > gpurun_out/rccl1_bench.log 2>&1 || exit $?
