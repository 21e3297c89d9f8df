#!/bin/bash
# rocprofv3 evidence for bench.py (run under gpurun):
#   1. --kernel-trace --stats of the default bench (average kernel durations)
#   2. --pmc FETCH_SIZE and 3. --pmc WRITE_SIZE passes (each on its own, kernel-trace only)
# then scripts/summarize_profile.py writes profiles/<tag>_*.csv|json.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r1}
WL=${WL:-c2}
OUT=gpurun_out/prof_$WL
mkdir -p $OUT
BENCH="bench.py --workload $WL --steps ${STEPS:-5} --warmup 1 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace \
    -- python3 $BENCH > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o fetch \
    -- python3 $BENCH --no-timing > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o write \
    -- python3 $BENCH --no-timing > $OUT/write.log 2>&1 || exit $?
PROFILES_DIR=$OUT/profiles python3 scripts/summarize_profile.py $OUT $WL $TAG > $OUT/summary.log 2>&1 || exit $?
