#!/bin/bash
# Band width sweep of the paged A stream kernel at C3 and C4 (tiled order); 0 = no bands.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/spmv_variants.py c3 30 3 A=26:4:262144:4,26:4:131072:4,26:4:524288:4,26:4:1048576:4,26:4:0:4 \
    > gpurun_out/c3_bands.log 2>&1 || exit $?
timeout -k 10 900 python -u scripts/spmv_variants.py c4 10 2 A=26:4:262144:4,26:4:524288:4,26:4:1048576:4,26:4:4194304:4,26:4:0:4 \
    > gpurun_out/c4_bands.log 2>&1 || exit $?
