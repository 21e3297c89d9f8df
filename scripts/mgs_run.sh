#!/bin/bash
# MGS experiment: GPU parity tests, benches with the one-workgroup sweep on/off, kernel stats.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -rf > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for s in 1 0; do
  HGM_MGS_SINGLE=$s timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --time-classes MGS > gpurun_out/b_single$s.log 2>&1 || exit $?
  echo "c2 single=$s $(grep -o '"value": [0-9.]*' gpurun_out/b_single$s.log | head -1) $(grep -o '"mgs_pass_sweep": {[^}]*}' gpurun_out/b_single$s.log)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b_c2.log 2>&1 || exit $?
echo "c2 default $(grep -o '"value": [0-9.]*' gpurun_out/b_c2.log | head -1)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mgs -o t -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_mgs.log 2>&1 || exit $?
python3 - <<'PY'
import csv,glob
f=glob.glob("gpurun_out/prof_mgs/**/*kernel_stats.csv",recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r["Calls"], round(float(r["AverageNs"])/1e3,2), r["Name"][:90])
PY
