#!/bin/bash
# Bench lines with the XCD-contiguous banded A (default now) vs without (tune-a 26:4).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/xcd_ab.jsonl
for rep in 1 2; do
  for t in "" "--tune-a 26:4"; do
    for W in c4 c3; do
      timeout -k 10 400 python -u bench.py --workload $W --no-cpu-baseline --steps 10 $t > gpurun_out/b.log 2>&1 || exit $?
      echo "{\"wl\": \"$W\", \"tune\": \"$t\", \"line\": $(tail -1 gpurun_out/b.log)}" >> gpurun_out/xcd_ab.jsonl
    done
  done
done
