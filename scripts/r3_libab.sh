#!/bin/bash
# A/B of experiment builds of libhgmres (HGM_LIB) on the C4 fused pass micro-benchmark (BENCH=1:
# the default C4 bench), alternating library / default twice.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3libab
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for lib in default $LIBS; do
    if [ $lib = default ]; then unset HGM_LIB; else export HGM_LIB=$PWD/exp/$lib; fi
    if [ "${BENCH:-0}" = 1 ]; then
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/$lib.$rep.log 2>&1 || { tail -20 $O/$lib.$rep.log; exit 1; }
      grep '^{' $O/$lib.$rep.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['roofline']['avg_launch_us'])"
    else
      timeout -k 10 300 python -u scripts/fused_micro.py 4096 47 20 ${VARIANTS:-w4r32g8d2p1} > $O/$lib.$rep.log 2>&1 || { tail -20 $O/$lib.$rep.log; exit 1; }
      grep '^{' $O/$lib.$rep.log | sed "s/^/$lib /"
    fi
  done
done
