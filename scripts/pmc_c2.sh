# PMC passes over the C2 bench (one counter group per run) -> gpurun_out/r4/pmc_c2k/
set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && O=gpurun_out/r4/pmc_c2k && mkdir -p $O
B="bench.py --workload ${WL:-c2} --steps 2 --warmup 1 --no-cpu-baseline --no-timing $*"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "FETCH_SIZE" "TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o p$i -- python3 $B > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; echo "pass $i failed"; break; }
done
python3 scripts/pmc_kernels.py $O/p1 $O/p2 $O/p3 $O/p4
