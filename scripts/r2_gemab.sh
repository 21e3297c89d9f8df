#!/bin/bash
# m-space Gram error monitor (AB *_bounds with B = A' on the device): parity tests, then C4.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 300 \
    --timeout-method thread -k "ab_gram or residual_monitor or golden or c4_ab or one_reduction or shard or null_x" \
    > gpurun_out/gemab_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/gemab_bench.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-cpu-baseline --steps 10 --opt gram_err=0 > gpurun_out/gemab_bench_off.log 2>&1 || exit $?
