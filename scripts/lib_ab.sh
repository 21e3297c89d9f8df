#!/bin/bash
# Alternating A/B of two library builds on the workloads' A and B products:
#   bash scripts/lib_ab.sh <old.so> <workload...>   (the in-tree build is "new")
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=$1; shift
: > gpurun_out/lib_ab.jsonl
for wl in "$@"; do
  for rep in 1 2; do
    HGM_LIB=$OLD timeout -k 10 300 python -u scripts/time_ops.py $wl >> gpurun_out/lib_ab.jsonl 2> gpurun_out/lib_ab.err || exit $?
    timeout -k 10 300 python -u scripts/time_ops.py $wl >> gpurun_out/lib_ab.jsonl 2> gpurun_out/lib_ab.err || exit $?
  done
done
