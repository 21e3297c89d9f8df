#!/bin/bash
# Counter passes on the C4 SpMV kernels (production choices: A banded stream, B stream), tiled order.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_spmv
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || exit $?
run() {  # name, counters
  timeout -s KILL 300 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $OUT/$1 -o $1 \
      -- python3 scripts/spmv_once.py c4 A:10:4 B:10:4 --reps 3 > $OUT/$1.log 2>&1
}
export HGM_SIDDON_TILE=4 HGM_SIDDON_SUPER=0
run tcp "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" || exit $?
run tcc "TCC_HIT_sum TCC_MISS_sum" || exit $?
run sq "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU" || exit $?
run ta "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" || exit $?
