#!/bin/bash
# 272-page fp64 budget as the default: paged / banded / dual SpMV tests and the default bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
    -k "dual_strip or banded or paged_stream or stream_spmv or c4 or fullsize or 4096" \
    --timeout 200 --timeout-method thread > gpurun_out/p272_tests.log 2>&1 || exit $?
echo "tests done"
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
