#!/bin/bash
# Bench lines of the non-default workloads (under gpurun), one log each under gpurun_out/.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "c3gcv:" "c3gcv:--orth cgs2" "c4:" "c5:" "c5m:"; do
  wl=${spec%%:*}; extra=${spec#*:}; tag=$wl${extra:+_cgs2}
  timeout -k 10 400 python bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline $extra \
      > gpurun_out/bench_$tag.log 2>&1 || { tail -20 gpurun_out/bench_$tag.log; exit 1; }
  grep '^{' gpurun_out/bench_$tag.log | tail -1 | cut -c1-160
done
