#!/bin/bash
# Evidence refresh (under gpurun): full GPU tests + smoke + C2 bench + rocprof/PMC (gpu_round.sh),
# then the C3 and C5 (LSQR / LSMR fp32) bench lines.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
SWEEP=0 bash scripts/gpu_round.sh || exit $?
for wl in c3 c5 c5m; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$wl.log 2>&1 || exit $?
done
