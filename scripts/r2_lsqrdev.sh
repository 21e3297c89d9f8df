#!/bin/bash
# GPU: device-resident LSQR scalars -- tests, then C5 A/B (lsqr_dev=1/0 alternating).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_parity_mode.py tests/test_gpu_fullsize.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -k "lsqr or golub or c5 or shard" > gpurun_out/lsqrdev_tests.log 2>&1 || exit $?
: > gpurun_out/lsqrdev_ab.jsonl
for rep in 1 2; do
  for f in 1 0; do
    timeout -k 10 400 python -u bench.py --workload c5 --no-cpu-baseline --steps 10 --opt lsqr_dev=$f > gpurun_out/b.log 2>&1 || exit $?
    echo "{\"lsqr_dev\": $f, \"line\": $(tail -1 gpurun_out/b.log)}" >> gpurun_out/lsqrdev_ab.jsonl
  done
done
