#!/bin/bash
# Alternating isolated-SpMV comparison of library builds (HGM_LIB):
#   LIBS="hgmres/libhgmres.so hgmres/libhgmres_old.so" CFG=c4 CASES=... OPS=A REPS=2 bash scripts/lib_sweep_compare.sh
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in $(seq ${REPS:-2}); do
  for lib in $LIBS; do
    HGM_LIB=$GRAFT_REPO_ROOT/hybrid-gmres_amd/$lib timeout -k 10 600 python scripts/spmv_sweep.py ${CFG:-c4} --tiles ${TILES:-4} \
        --cases $CASES --ops ${OPS:-A} --reps ${SREPS:-10} > gpurun_out/lsc.log 2>&1 || { tail -5 gpurun_out/lsc.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/lsc.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$lib', d['cfg'], d['op'], d['band_w'], d['group'], d['variant'], d['avg_us'], d['GBps'])"
  done
done
