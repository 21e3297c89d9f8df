#!/bin/bash
# Closing evidence for the final code: GPU suite, smoke, default bench + its kernel trace, the
# C4 profile (trace + FETCH/WRITE traffic), and a 2-rank sharded C4 bench launched like the
# driver's N=2 run (host all-reduce, both ranks on the one GPU of this box).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/r2_final.sh || exit $?
echo "final done"
TAG=r2 WL=c4 STEPS=3 bash scripts/profile_bench.sh || exit $?
echo "profile done"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --comm host --same-device --no-cpu-baseline \
    > gpurun_out/shard2_emulated.log 2>&1 || exit $?
echo "shard2 done"
