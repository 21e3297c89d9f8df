#!/bin/bash
# C2 SpMV kernel choices: row kernels (default) vs the paged streaming kernel.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/spmv_variants.py c2 50 3 A=1:16,26:4,26:8,24:4,10:4 B=0:8,26:4,26:8,24:4,10:4 \
    > gpurun_out/c2_spmv_variants.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/spmv_variants.py c3 20 2 A=10:4,26:4 B=10:4,26:4,26:8 \
    > gpurun_out/c3_spmv_variants.log 2>&1 || exit $?
