#!/bin/bash
# Counter passes on the C4 stream SpMV kernels, unpaged (10:4) then paged (26:4), fp64 and fp32,
# tiled order (the production choice); then FETCH/WRITE traffic of the C3 and C5 bench lines.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_paged
mkdir -p $OUT
run() {  # name, counters
  timeout -s KILL 300 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $OUT/$1 -o $1 \
      -- python3 scripts/spmv_once.py c4 A:10:4 A:26:4 B:10:4 B:26:4 --reps 3 > $OUT/$1.log 2>&1
}
export HGM_SIDDON_TILE=4 HGM_SIDDON_SUPER=0
for DT in f64 f32; do
  export HGM_DTYPE=$DT
  run sq_$DT "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU" || exit $?
  run ta_$DT "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" || exit $?
  run fetch_$DT "FETCH_SIZE" || exit $?
done
unset HGM_DTYPE HGM_SIDDON_TILE HGM_SIDDON_SUPER
TAG=r2 WL=c5 STEPS=2 bash scripts/profile_bench.sh || exit $?
TAG=r2 WL=c3 STEPS=3 bash scripts/profile_bench.sh || exit $?
