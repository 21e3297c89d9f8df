#!/bin/bash
# rocprof kernel trace + FETCH/WRITE traffic of the default C4 command and of the C3 line.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=r2 WL=c4 STEPS=3 bash scripts/profile_bench.sh || exit $?
TAG=r2 WL=c3 STEPS=3 bash scripts/profile_bench.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
