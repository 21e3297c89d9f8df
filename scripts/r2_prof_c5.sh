#!/bin/bash
# rocprof kernel trace + FETCH/WRITE traffic of the C5 LSQR / LSMR lines (two-round fp32 staging).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r2 WL=c5 STEPS=3 bash scripts/profile_bench.sh || exit $?
TAG=r2 WL=c5m STEPS=3 bash scripts/profile_bench.sh || exit $?
