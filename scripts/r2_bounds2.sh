#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bounds.py tests/test_mex_gateway.py -m gpu -x -q -s --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_bounds2.log 2>&1 || exit $?
timeout -k 10 600 python -u scripts/bounds_scale.py 512 30 20 60 > gpurun_out/bounds_scale_c2.log 2>&1 || exit $?
