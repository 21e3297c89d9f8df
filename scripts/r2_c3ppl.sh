#!/bin/bash
# C3 MGS sweep granularity: element pairs per lane of the dots (mgs1_ppl) and update (mgs_ppl) passes.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/c3ppl.jsonl
for rep in 1 2; do
  for o in "mgs1_ppl=2" "mgs1_ppl=1" "mgs1_ppl=4" "mgs_ppl=2" "mgs_ppl=4"; do
    timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --steps 10 --time-classes MGS --opt $o > gpurun_out/c3ppl_one.log 2>&1 || exit $?
    echo "{\"opt\": \"$o\", \"line\": $(tail -1 gpurun_out/c3ppl_one.log)}" >> gpurun_out/c3ppl.jsonl
  done
done
