#!/bin/bash
# Side dot x_true'(B*q) in the row-wave pass: the tests that exercise the m-space Gram error
# monitor (single rank, one-rank RCCL, fused kernels, C4 fixture), the default bench, and the
# 2-rank sharded bench emulated on the one GPU (host all-reduce).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3zx
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_rccl.py tests/test_gpu_fullsize.py::test_c4_ab_gmres_full_size \
    "tests/test_gpu_parity.py" -k "fused or rccl or c4 or gram or ab or shard or dist" -m gpu -q -rA --timeout 600 --timeout-method thread > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | cut -c1-400
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 5 --warmup 1 --comm host --same-device --no-cpu-baseline > $O/shard2.log 2>&1 || { tail -20 $O/shard2.log; exit 1; }
grep '^{' $O/shard2.log | tail -1 | cut -c1-600
timeout -k 10 300 python bench.py --gpus 1 --shard1 --steps 5 --warmup 1 --no-cpu-baseline > $O/shard1_rccl.log 2>&1 || { tail -20 $O/shard1_rccl.log; exit 1; }
grep '^{' $O/shard1_rccl.log | tail -1 | cut -c1-300
