#!/bin/bash
# Dual-strip bands (HGM_OPT_BAND_DUAL): parity test, then alternating C4 bench runs on/off.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "dual_strip or banded or paged_stream" \
    --timeout 120 --timeout-method thread > gpurun_out/dual_tests.log 2>&1 || exit $?
for i in 1 2; do
  for d in 1 0; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --opt band_dual=$d \
        > gpurun_out/dual_bench_$d.$i.log 2>&1 || exit $?
    tail -1 gpurun_out/dual_bench_$d.$i.log >> gpurun_out/dual_ab.jsonl
    echo "band_dual=$d run $i done"
  done
done
