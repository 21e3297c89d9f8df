#!/bin/bash
# fp64 page budget 272 vs 256 with dual strips (isolated C4/C3 A and B products), then the C5m
# (LSMR fp32) bench line with dual strips.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/lib_ab.sh exp/lib_p272.so c4 c3 || exit $?
echo "lib ab done"
timeout -k 10 300 python -u bench.py --workload c5m --no-cpu-single > gpurun_out/c5m.log 2>&1 || exit $?
