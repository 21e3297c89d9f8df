#!/bin/bash
# GPU: fused one-reduction MGS (solve folded into the update) -- bitwise tests, then A/B benches.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "mgs_fused or one_reduction or gram_error" > gpurun_out/fused_tests.log 2>&1 || exit $?
: > gpurun_out/fused_ab.jsonl
for rep in 1 2 3; do
  for f in 1 0; do
    for W in c2 c3; do
      timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline --opt mgs_fused=$f --time-classes MGS \
          > gpurun_out/b.log 2>&1 || exit $?
      echo "{\"wl\": \"$W\", \"fused\": $f, \"line\": $(tail -1 gpurun_out/b.log)}" >> gpurun_out/fused_ab.jsonl
    done
  done
done
