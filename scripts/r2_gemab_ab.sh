#!/bin/bash
# C4 alternating runs: Gram monitor (recon on the aux stream), Gram monitor with the residual
# recon serialised on the main stream, explicit reconstruction.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/gemab_ab.jsonl
for rep in 1 2; do
  for opt in "gram_err=1" "recon_serial=1" "gram_err=0"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --opt $opt > gpurun_out/gemab_one.log 2>&1 || exit $?
    echo "{\"opt\": \"$opt\", \"line\": $(tail -1 gpurun_out/gemab_one.log)}" >> gpurun_out/gemab_ab.jsonl
  done
done
