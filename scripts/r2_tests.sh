#!/bin/bash
# GPU test suite + parity-mode report (run under gpurun).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
HGM_PARITY_REPORT=gpurun_out/parity_mode.json timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q -rA \
    --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
exit $rc
