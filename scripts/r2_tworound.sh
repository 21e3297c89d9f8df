#!/bin/bash
# Two-round LDS page staging (fp32): paged-kernel bitwise tests, then C5 / C4 against the
# previous build (exp/lib_base.so).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "paged or stream_spmv or banded or lsqr or lsmr" > gpurun_out/tworound_tests.log 2>&1 || exit $?
bash scripts/lib_ab.sh exp/lib_base.so c5 c4 || exit $?
