#!/bin/bash
# Round-3 closing evidence: GPU suite, smoke, default C4 bench + its rocprof kernel trace, the
# side-workload lines (C2, C3, C3-GCV MGS/CGS2, C5, C5m), and the 2-rank sharded C4 bench emulated on
# the one GPU.  Each GPU step under its own time limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 300 --timeout-method thread \
    > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
grep '^{' $O/bench_default.log | tail -1 | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace \
    -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
for W in c5 c5m c3 c3gcv c2; do
  timeout -k 10 300 python -u bench.py --workload $W --no-cpu-single > $O/bench_$W.log 2>&1 || { tail -20 $O/bench_$W.log; exit 1; }
  grep '^{' $O/bench_$W.log | tail -1 | cut -c1-120
done
timeout -k 10 300 python -u bench.py --workload c3gcv --orth cgs2 --no-cpu-baseline > $O/bench_c3gcv_cgs2.log 2>&1 || exit 1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 5 --warmup 1 --comm host --same-device --no-cpu-baseline > $O/shard2.log 2>&1 || { tail -20 $O/shard2.log; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --shard1 --steps 5 --warmup 1 --no-cpu-baseline > $O/shard1_rccl.log 2>&1 || { tail -20 $O/shard1_rccl.log; exit 1; }
echo r3_final done
