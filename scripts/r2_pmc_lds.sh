#!/bin/bash
# LDS counters of the production C4 stream kernels (A: paged + XCD order 30:4, B: paged 26:4), fp64.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_lds
mkdir -p $OUT
export HGM_SIDDON_TILE=4 HGM_SIDDON_SUPER=0
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_ADDR_CONFLICT SQ_BUSY_CYCLES SQ_WAVES \
    --kernel-trace --output-format csv -d $OUT/lds -o lds -- python3 scripts/spmv_once.py c4 A:30:4 B:26:4 --reps 3 > $OUT/lds.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VALU \
    --kernel-trace --output-format csv -d $OUT/sq -o sq -- python3 scripts/spmv_once.py c4 A:30:4 B:26:4 --reps 3 > $OUT/sq.log 2>&1 || exit $?
