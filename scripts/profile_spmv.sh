#!/bin/bash
# rocprofv3 passes for the SpMV kernels (run under gpurun).  Each counter group in
# its own pass, kernel-trace only alongside (no sys/runtime trace with --pmc).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
CASES_C4="A:1:32 A:2:32 A:6:32 B:1:8 B:0:16"
CASES_C2="A:1:32 B:0:8"
run() {  # name, counters, cfg, cases...
  local name=$1 ctrs=$2 cfg=$3; shift 3
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/$name -o $name \
      -- python3 scripts/spmv_once.py $cfg "$@" > $OUT/$name.log 2>&1
}
run c4_fetch FETCH_SIZE c4 $CASES_C4 || exit $?
run c4_write WRITE_SIZE c4 $CASES_C4 || exit $?
run c4_tcc "TCC_HIT_sum TCC_MISS_sum" c4 $CASES_C4 || exit $?
run c2_fetch FETCH_SIZE c2 $CASES_C2 || exit $?
# bench kernel-trace summary (average kernel durations to cross-check bench.py's HIP-event numbers)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_trace -o bench \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_trace.log 2>&1 || exit $?
