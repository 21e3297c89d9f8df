#!/bin/bash
# Alternating isolated SpMV timings of library builds:
#   bash scripts/lib_sweep.sh <workload> <lib.so> [<lib.so> ...]   (two rounds)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
WL=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    HGM_LIB=$lib timeout -k 10 300 python -u scripts/time_ops.py $WL >> gpurun_out/lib_sweep.jsonl 2> gpurun_out/lib_sweep.err || exit $?
  done
done
