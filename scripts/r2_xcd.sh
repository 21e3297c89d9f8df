#!/bin/bash
# XCD-contiguous chunk order (variant bit 4) for the paged stream kernels at C4 and C3.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/spmv_variants.py c4 10 3 A=26:4,30:4 B=26:4,30:4 > gpurun_out/c4_xcd.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/spmv_variants.py c3 30 3 A=26:4,30:4 B=26:4,30:4 > gpurun_out/c3_xcd.log 2>&1 || exit $?
