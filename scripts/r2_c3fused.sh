#!/bin/bash
# C3: MGS solve fused into the update prologue (default) vs its own launch (mgs_fused=0).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/c3fused.jsonl
for rep in 1 2; do
  for o in "mgs_fused=1" "mgs_fused=0"; do
    timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --steps 10 --time-classes MGS --opt $o > gpurun_out/c3f_one.log 2>&1 || exit $?
    echo "{\"opt\": \"$o\", \"line\": $(tail -1 gpurun_out/c3f_one.log)}" >> gpurun_out/c3fused.jsonl
  done
done
