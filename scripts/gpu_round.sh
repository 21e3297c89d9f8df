#!/bin/bash
# Full GPU round under gpurun: parity tests, smoke, bench, rocprof evidence for the bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_check.sh || exit $?
SWEEP=0 bash scripts/profile_bench.sh || exit $?
