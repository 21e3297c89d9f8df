#!/bin/bash
# Round-2 evidence refresh: -m gpu suite, smoke, default bench (C4 + cpu_baseline), side lines,
# rocprof + FETCH/WRITE of the default command.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/r2_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
for W in c2 c3 c3gcv c5 c5m; do
  timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline > gpurun_out/bench_$W.log 2>&1 || exit $?
done
TAG=r2 WL=c4 STEPS=3 bash scripts/profile_bench.sh || exit $?
