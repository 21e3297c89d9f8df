#!/bin/bash
# GPU tests, the default bench line (C4, with cpu_baseline), and rocprof evidence of that command.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/r2_tests.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
TAG=r2 WL=c4 STEPS=3 bash scripts/profile_bench.sh || exit $?
