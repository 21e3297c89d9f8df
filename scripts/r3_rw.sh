#!/bin/bash
# Row-wave fused pass (kind 1): fused parity tests, then the C4 micro-benchmark of A*(B*q)
# against the two-pass form and the sub-chunk pass.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3rw
mkdir -p $O
export HGM_FUSED_VERBOSE=1
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -m gpu -q -rA --timeout 300 --timeout-method thread \
      > $O/tests.log 2>&1; echo "tests rc=$?"; grep -E "passed|failed|FAILED|Error" $O/tests.log | tail -12
fi
timeout -k 10 600 python -u scripts/fused_micro.py 4096 47 20 ${VARIANTS:-two,f1024,w4r32g4,w4r32g8,w2r32g4,w2r24g4,w1r16g4,w4r24g4} \
    > $O/micro.log 2>&1 || { tail -30 $O/micro.log; exit 1; }
cat $O/micro.log
