#!/bin/bash
# rocprofv3 PMC passes for the C4 SpMV kernels in the column-major and tiled pixel orders
# (run under gpurun; one counter group per pass, kernel-trace only alongside).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_c4
mkdir -p $OUT
run() {  # name, counters, tile, super, cases...
  local name=$1 ctrs=$2
  export HGM_SIDDON_TILE=$3 HGM_SIDDON_SUPER=$4
  shift 4
  timeout -k 10 400 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d $OUT/$name -o $name \
      -- python3 scripts/spmv_once.py c4 "$@" > $OUT/$name.log 2>&1
}
CM="A:8:32:131072:8 A:1:32 B:8:8 B:0:8"
TL="A:8:16:262144:8 A:1:32 B:8:4"
run cm_fetch FETCH_SIZE 1 0 $CM || exit $?
run cm_write WRITE_SIZE 1 0 $CM || exit $?
run cm_sq "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD" 1 0 $CM || exit $?
run tl_fetch FETCH_SIZE 4 256 $TL || exit $?
run tl_tcc "TCC_HIT_sum TCC_MISS_sum" 4 256 $TL || exit $?
run tl_sq "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD" 4 256 $TL || exit $?
