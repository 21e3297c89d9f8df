#!/bin/bash
# Band widths with the XCD-contiguous chunk order.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u scripts/spmv_variants.py c4 10 2 A=30:4:262144:4,30:4:131072:4,30:4:524288:4,30:4:393216:4 > gpurun_out/c4_bands3.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/spmv_variants.py c3 30 3 A=30:4:131072:4,30:4:65536:4,30:4:262144:4,30:4:196608:4 > gpurun_out/c3_bands3.log 2>&1 || exit $?
