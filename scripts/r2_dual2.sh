#!/bin/bash
# Dual strips incl. pixel shards: band/shard/RCCL tests, then alternating on/off bench runs of
# C3, C5 and the one-rank RCCL sharded C4 (--shard1).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rccl.py -m gpu -x -q \
    -k "dual_strip or banded or paged_stream or shard or rccl" \
    --timeout 200 --timeout-method thread > gpurun_out/dual2_tests.log 2>&1 || exit $?
echo "tests done"
for i in 1 2; do
  for d in 1 0; do
    for w in c3 c5; do
      timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 2 --opt band_dual=$d \
          > gpurun_out/dual2_$w.$d.$i.log 2>&1 || exit $?
      echo "{\"w\": \"$w\", \"band_dual\": $d, \"line\": $(tail -1 gpurun_out/dual2_$w.$d.$i.log)}" >> gpurun_out/dual2_ab.jsonl
    done
    timeout -k 10 300 python -u bench.py --shard1 --no-cpu-baseline --steps 10 --warmup 2 --opt band_dual=$d \
        > gpurun_out/dual2_s1.$d.$i.log 2>&1 || exit $?
    echo "{\"w\": \"c4shard1\", \"band_dual\": $d, \"line\": $(tail -1 gpurun_out/dual2_s1.$d.$i.log)}" >> gpurun_out/dual2_ab.jsonl
    echo "band_dual=$d run $i done"
  done
done
