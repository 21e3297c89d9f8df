#!/bin/bash
# C3 bench lines after the band-width change + the C3 full-size tests.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c3" \
    > gpurun_out/c3_tests.log 2>&1 || exit $?
for W in c3 c3gcv c3 c3gcv; do
  timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline > gpurun_out/bench_$W.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$W.log >> gpurun_out/c3_bench.jsonl
done
