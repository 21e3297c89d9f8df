#!/bin/bash
# rocprofv3 of the C4 bench with the row-wave fused pass: kernel trace + stats, then PMC passes
# (one counter group per run, each under its own time limit).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3pmcrw
mkdir -p $O
BENCH="bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace \
    -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline $EXTRA > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep '^{' $O/trace.log | tail -1
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o p$i \
      -- python3 $BENCH > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python3 scripts/pmc_fused_summary.py $O $O/summary.json
echo pmc done
