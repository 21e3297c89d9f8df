#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_edge.py tests/test_gpu_parity_mode.py tests/test_gpu_bounds.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/edge_tests.log 2>&1 || exit $?
