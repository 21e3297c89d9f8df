#!/bin/bash
# C5 LSQR / LSMR bench lines (fp32 operator) with the all-core CPU baseline.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload c5 > gpurun_out/bench_c5.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --workload c5m > gpurun_out/bench_c5m.log 2>&1 || exit $?
