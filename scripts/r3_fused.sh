#!/bin/bash
# Fused A*(B*q): parity tests, then the C4 bench with the pass off and on (option fused_ab, same
# library) and its workgroup-size / prefetch variants.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py::test_c4_ab_gmres_full_size \
      -m gpu -q -rA --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
run() {   # tag, bench options
  local tag=$1; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > $O/bench_$tag.log 2>&1 || { tail -20 $O/bench_$tag.log; exit 1; }
  grep '^{' $O/bench_$tag.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; k=d['kernels'].get('spmv_AB_fused',{}); print('$tag', d['value'], r['kernel'], r['avg_launch_us'], r['achieved'], k.get('effective_GBps_two_pass'))"
}












run off --opt fused_ab=0
run bs1024 --opt fused_ab=1
run d1 --opt fused_ab=1 --opt fused_dbg=1
run d2 --opt fused_ab=1 --opt fused_dbg=2
run d4 --opt fused_ab=1 --opt fused_dbg=4
run d8 --opt fused_ab=1 --opt fused_dbg=8
run d15 --opt fused_ab=1 --opt fused_dbg=15
echo r3_fused done
