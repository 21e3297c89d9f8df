#!/bin/bash
# GPU: filter-factor bounds + analyze_regularization pipeline tests.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bounds.py tests/test_mex_gateway.py -m gpu -x -v -s --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_bounds.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_bounds.log
exit $rc
