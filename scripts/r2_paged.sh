#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "paged or stream_spmv or banded" --timeout 120 --timeout-method thread > gpurun_out/paged_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/spmv_ab.py c4 20 > gpurun_out/spmv_ab_c4.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/spmv_ab.py c4 20 f32 > gpurun_out/spmv_ab_c4f32.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/spmv_ab.py c3 50 > gpurun_out/spmv_ab_c3.log 2>&1 || exit $?
