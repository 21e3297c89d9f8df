#!/bin/bash
# Side-line bench lines (C2, C3, C3-GCV MGS/CGS2, C5) with the final kernels.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for W in c5 c3 c3gcv c2; do
  timeout -k 10 300 python -u bench.py --workload $W --no-cpu-single > gpurun_out/bench_$W.log 2>&1 || exit $?
  echo "$W done"
done
timeout -k 10 300 python -u bench.py --workload c3gcv --orth cgs2 --no-cpu-baseline > gpurun_out/bench_c3gcv_cgs2.log 2>&1 || exit $?
