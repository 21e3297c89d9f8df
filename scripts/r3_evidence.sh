#!/bin/bash
# Round-3 evidence (under gpurun): GPU tests, smoke, the driver's default bench line, and the
# rocprofv3 kernel-trace summary of the same bench command (A and B stream kernels are separate
# instantiations since round 3).  Each GPU step under its own time limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
TESTS=${TESTS:-tests}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu ${PYX:--x} -q -rA --timeout 300 --timeout-method thread \
      > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
  grep '^{' $O/bench_default.log | tail -1
fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace \
      -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
  grep '^{' $O/trace.log | tail -1
fi
echo r3_evidence done
