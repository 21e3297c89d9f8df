#!/bin/bash
# A/B a runtime switch on the bench: for each setting in $SETS ("VAR=val VAR2=val ..."; sets
# separated by ';'), one bench line per workload in $WLS with all kernel classes timed.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
IFS=';' read -ra S <<< "${SETS:-HGM_MGS_FORM=1;HGM_MGS_FORM=0}"
for w in ${WLS:-c2}; do
  for s in "${S[@]}"; do
    timeout -k 10 300 env $s python bench.py --workload $w --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
        --time-classes ${CLASSES:-ALL} $BARGS > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/ab.log') if l.startswith('{')][-1])
print('$w [$s]', d['value'], {k: round(v['avg_us'],2) for k,v in d['kernels'].items()})"
  done
done
