#!/bin/bash
# Band reduction with eight loads in flight: C4 bench A (band reduce inside the A class) vs the
# previous build, alternating.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/bandred.jsonl
for rep in 1 2; do
  for lib in exp/lib_base.so hybrid-gmres_amd/hgmres/libhgmres.so; do
    HGM_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 > gpurun_out/bandred_one.log 2>&1 || exit $?
    echo "{\"lib\": \"$lib\", \"line\": $(tail -1 gpurun_out/bandred_one.log)}" >> gpurun_out/bandred.jsonl
  done
done
