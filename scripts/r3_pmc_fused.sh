#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) on the C4 bench with the fused A*(B*q) pass.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3pmc
mkdir -p $O
BENCH="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-timing --opt fused_ab=1 --opt fused_bs=${FBS:-1024} $EXTRA"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o p$i \
      -- python3 $BENCH > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
echo pmc done
