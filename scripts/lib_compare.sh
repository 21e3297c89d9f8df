#!/bin/bash
# Alternating comparison of experiment library builds (HGM_LIB) on one workload:
#   LIBS="hgmres/libhgmres.so hgmres/libhgmres_u4.so" WL=c2 REPS=3 bash scripts/lib_compare.sh
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in $(seq ${REPS:-3}); do
  for lib in $LIBS; do
    HGM_LIB=$GRAFT_REPO_ROOT/hybrid-gmres_amd/$lib timeout -k 10 300 python bench.py --workload ${WL:-c2} --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline $BARGS > gpurun_out/lc.log 2>&1 || { tail -5 gpurun_out/lc.log; exit 1; }
    echo "$lib $(grep -o '"value": [0-9.]*' gpurun_out/lc.log | head -1) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/lc.log)"
  done
done
