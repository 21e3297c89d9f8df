#!/bin/bash
# Quick GPU iteration: parity tests (TESTS=0 skips), then one bench line per workload in
# $WLS (default c2) plus the MGS class timing of C2.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
fi
for w in ${WLS:-c2}; do
  timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline $BARGS > gpurun_out/q_$w.log 2>&1 || { tail -20 gpurun_out/q_$w.log; exit 1; }
  echo "$w $(grep -o '"value": [0-9.]*' gpurun_out/q_$w.log | head -1) $(grep -o '"roofline": {[^}]*}' gpurun_out/q_$w.log | cut -c1-160)"
done
if [ "${MGS:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --time-classes ALL > gpurun_out/q_all.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/q_all.log') if l.startswith('{')][-1])
print('c2 ALL-timed', d['value'], {k: round(v['avg_us'],2) for k,v in d['kernels'].items()})"
fi
