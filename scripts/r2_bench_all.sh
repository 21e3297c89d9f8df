#!/bin/bash
# GPU tests + bench lines for every workload (side lines use --no-cpu-baseline).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/r2_tests.sh || exit $?
for W in c4 c5 c5m c3 c3gcv c2; do
  timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline > gpurun_out/bench_$W.log 2>&1 || exit $?
done
