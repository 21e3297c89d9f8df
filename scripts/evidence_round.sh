#!/bin/bash
# Evidence refresh (under gpurun): full GPU tests + smoke + C2 bench + rocprof/PMC (gpu_round.sh),
# then the C3 bench line.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
SWEEP=0 bash scripts/gpu_round.sh || exit $?
timeout -k 10 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit $?
