#!/bin/bash
# C5 LSQR / LSMR kernel traces: where the time between the SpMVs goes.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in c5 c5m; do
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps_$wl -o trace \
    -- python3 bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-timing > gpurun_out/gaps_$wl.log 2>&1 || exit $?
done
