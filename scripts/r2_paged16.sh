#!/bin/bash
# C3 B (55,043 columns: 16-bit indices) with and without the paged gathers, A/B bench lines.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/paged16_ab.jsonl
for rep in 1 2; do
  for f in 1 0; do
    timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline --opt paged16=$f --time-classes AB > gpurun_out/b.log 2>&1 || exit $?
    echo "{\"paged16\": $f, \"line\": $(tail -1 gpurun_out/b.log)}" >> gpurun_out/paged16_ab.jsonl
  done
done
