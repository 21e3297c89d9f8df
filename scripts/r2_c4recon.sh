#!/bin/bash
# C4: reconstruction on the aux stream (recon_serial=0) vs serialised (default at n >= 4 Mi).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/c4_recon_ab.jsonl
for rep in 1 2; do
  for r in 1 0; do
    timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 10 --opt recon_serial=$r --time-classes AB \
        > gpurun_out/b.log 2>&1 || exit $?
    echo "{\"recon_serial\": $r, \"line\": $(tail -1 gpurun_out/b.log)}" >> gpurun_out/c4_recon_ab.jsonl
  done
done
