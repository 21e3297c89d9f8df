#!/bin/bash
# rocprof kernel trace + FETCH/WRITE traffic of C4 (default), C3 and C5 with the dual strips.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in c4 c3 c5; do
  TAG=r2 WL=$w STEPS=3 bash scripts/profile_bench.sh || exit $?
  echo "$w profiled"
done
