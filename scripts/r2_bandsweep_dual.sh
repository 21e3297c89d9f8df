#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in c4 c3 c5; do
  timeout -k 10 400 python -u scripts/band_sweep_dual.py $w >> gpurun_out/bandsweep_dual.jsonl 2> gpurun_out/bandsweep_dual.err || exit $?
done
