#!/bin/bash
# The RCCL transport on one GPU (one-rank communicator): parity tests, then the C4 solve on the
# sharded code path next to the default single-context line.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/rccl1_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --shard1 --no-cpu-baseline --steps 10 > gpurun_out/rccl1_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/rccl1_bench_plain.log 2>&1 || exit $?
