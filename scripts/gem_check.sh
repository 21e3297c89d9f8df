#!/bin/bash
# Gram error monitor check (under gpurun): parity tests of the GMRES family, then A/B bench
# HGM_GRAM_ERR=0/1 at C2 and C3 (alternating, same box).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "gram_error or c2_hybrid or one_reduction or golden or tol_stop or breakdown or residual_monitor or determinism" \
    > gpurun_out/gem_tests.log 2>&1 || { tail -30 gpurun_out/gem_tests.log; exit 1; }
tail -3 gpurun_out/gem_tests.log
V=$'HGM_GRAM_ERR=0 | \nHGM_GRAM_ERR=1 | \nHGM_GRAM_ERR=0 | \nHGM_GRAM_ERR=1 | '
VARIANTS="$V" bash scripts/ab_bench.sh || exit 1
WL=c3 STEPS=10 VARIANTS="$V" bash scripts/ab_bench.sh || exit 1
