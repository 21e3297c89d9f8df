#!/bin/bash
# GPU check (used with gpurun): parity tests, smoke, short bench, SpMV variant sweep.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 || exit $?
if [ "${SWEEP:-1}" = "1" ]; then
  timeout -k 10 600 python scripts/spmv_sweep.py ${SWEEP_CFGS:-c2 c3 c4} > gpurun_out/sweep.log 2>&1 || exit $?
fi
