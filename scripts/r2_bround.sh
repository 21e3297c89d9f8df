#!/bin/bash
# fp32 B with one LDS round again (page index limit per operator): C5 against the previous build,
# then the paged-kernel tests.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "paged or stream_spmv or banded" > gpurun_out/bround_tests.log 2>&1 || exit $?
: > gpurun_out/lib_sweep.jsonl
bash scripts/lib_sweep.sh c5 exp/lib_base.so hybrid-gmres_amd/hgmres/libhgmres.so || exit $?
