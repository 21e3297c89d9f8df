#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
HGM_DTYPE=f32 timeout -k 10 600 python -u scripts/spmv_variants.py c4 10 2 A=30:4,26:4 B=26:4 > gpurun_out/c5_iso.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu-baseline --time-classes AB > gpurun_out/bench_c5ab.log 2>&1 || exit $?
