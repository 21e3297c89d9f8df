#!/bin/bash
# Round-2 first GPU call: smoke, default bench (C4), rocprof evidence of C4 before changes.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_c4.log 2>&1 || exit $?
TAG=r2pre WL=c4 STEPS=3 bash scripts/profile_bench.sh || exit $?
