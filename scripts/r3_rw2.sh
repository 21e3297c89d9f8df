#!/bin/bash
# Row-wave fused pass as the default: fused parity tests, the C4 20-iteration fixture test, and
# the default bench line.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3rw2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py::test_c4_ab_gmres_full_size -m gpu -q -rA \
    --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
grep -E "^\[fused" $O/tests.log | head -30
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1
