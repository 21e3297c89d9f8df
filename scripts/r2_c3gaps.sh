#!/bin/bash
# C3 kernel trace: the time between the SpMVs of the BA-RTP solve.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps_c3 -o trace \
  -- python3 bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline --no-timing > gpurun_out/gaps_c3.log 2>&1 || exit $?
