#!/bin/bash
# MGS update pass with eight column loads in flight: C3 and C2 benches (MGS class timed) against
# the previous build, alternating, then the MGS parity tests.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/mgsu8.jsonl
for wl in c3 c2; do
  for rep in 1 2; do
    for lib in exp/lib_base.so hybrid-gmres_amd/hgmres/libhgmres.so; do
      HGM_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --steps 10 --time-classes MGS > gpurun_out/mgsu8_one.log 2>&1 || exit $?
      echo "{\"lib\": \"$lib\", \"wl\": \"$wl\", \"line\": $(tail -1 gpurun_out/mgsu8_one.log)}" >> gpurun_out/mgsu8.jsonl
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "mgs or gram or golden" > gpurun_out/mgsu8_tests.log 2>&1 || exit $?
