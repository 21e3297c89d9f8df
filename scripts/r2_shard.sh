#!/bin/bash
# Tiled stored-order shards: the 2-rank emulation test, then the sharded C4 bench emulated as two
# ranks on the one GPU (host all-reduce): its monitors must match the single-rank solve.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 500 --timeout-method thread \
    -k "shard_emulation" > gpurun_out/shard_tests.log 2>&1 || exit $?
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 3 --warmup 1 --comm host --same-device --no-timing > gpurun_out/shard_bench.log 2>&1 || exit $?
