#!/bin/bash
# Narrower bands for the paged A stream kernel at C3 and C4.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/spmv_variants.py c3 30 3 A=26:4:131072:4,26:4:65536:4,26:4:32768:4,26:4:131072:8 \
    > gpurun_out/c3_bands2.log 2>&1 || exit $?
timeout -k 10 900 python -u scripts/spmv_variants.py c4 10 2 A=26:4:262144:4,26:4:131072:4,26:4:65536:4,26:4:32768:4 \
    > gpurun_out/c4_bands2.log 2>&1 || exit $?
