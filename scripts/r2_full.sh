#!/bin/bash
# Full GPU checkpoint: the -m gpu suite, smoke(), the default bench line.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/r2_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
