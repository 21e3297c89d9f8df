#!/bin/bash
# GPU recipes (run on the MI355X box under gpurun, from the repo root):
#     gpurun -- 'bash scripts/gpu.sh <recipe> [args]'
# Every GPU step runs under its own time limit and the recipe stops at the first failure.
# Outputs go to gpurun_out/$TAG/ (TAG defaults to r4); the file each recipe writes is the one
# copied to profiles/ under the name given below (profiles/README.md lists them).
#
#   evidence                 GPU tests, smoke, the default bench line, the rocprofv3 kernel-trace
#                            summary of the same command
#                            -> $TAG_gpu_tests.log, $TAG_bench_default_c4.json, $TAG_default_kernel_stats.csv
#   tests [PYTEST_ARGS]      pytest -m gpu (e.g. tests/test_gpu_fused.py -k gkb) -> $TAG_gpu_tests_<n>.log
#   bench WL [BENCH_ARGS]    one bench line of workload WL (c2 c3 c3gcv c4 c5 c5m) -> $TAG_bench_<wl>.json
#   trace WL [BENCH_ARGS]    rocprofv3 --kernel-trace --stats of that bench -> $TAG_<wl>_kernel_stats.csv
#   traffic WL [BENCH_ARGS]  FETCH_SIZE / WRITE_SIZE passes (one counter per run) + the per-kernel
#                            HBM-bytes summary (gfx950 x2 FETCH correction) -> traffic_<NAME or wl>.json
#                            (NAME=c4_unmatched with --unmatched: bench.py reads that file then)
#   pmc WL                   SQ / LDS counter groups of the fused pass, one run each
#                            -> $TAG_pmc_<wl>/summary.json
#   micro N ANGLES VARIANTS  hgm_spmv_ab micro-benchmark (scripts/fused_micro.py; F32=1 for fp32)
#                            -> $TAG_micro_<f32|f64>.jsonl
#   ab ROUNDS "ARGS_1" "ARGS_2" ...  alternating bench lines, one per argument set and round
#                            -> $TAG_ab.jsonl
#   libab OLD.so WL...       alternating library builds (HGM_LIB) on scripts/time_ops.py -> $TAG_lib_ab.jsonl
#   shardbudget [N...]       rocprofv3 kernel trace of the C4 solve on rank 0's shard of an N-way cut
#                            (default 2 4 8) -> $TAG_c4_shard_of<N>_kernel_stats.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r6}
O=gpurun_out/$TAG
mkdir -p "$O"
recipe=$1
shift

bench_line() {   # last JSON line of a log
  grep '^{' "$1" | tail -1
}

case "$recipe" in
  evidence)
    timeout -k 10 1500 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread \
        > "$O/${TAG}_gpu_tests.log" 2>&1 || { tail -40 "$O/${TAG}_gpu_tests.log"; exit 1; }
    tail -3 "$O/${TAG}_gpu_tests.log"
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit 1
    timeout -k 10 600 python bench.py --gpus 1 > "$O/bench_default.log" 2>&1 || { tail -20 "$O/bench_default.log"; exit 1; }
    bench_line "$O/bench_default.log" > "$O/${TAG}_bench_default_c4.json"
    cat "$O/${TAG}_bench_default_c4.json"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_default" -o trace \
        -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$O/trace_default.log" 2>&1 || exit 1
    bench_line "$O/trace_default.log" > "$O/${TAG}_bench_default_c4_traced.json"
    cp "$(find "$O/trace_default" -name '*kernel_stats.csv' | head -1)" "$O/${TAG}_default_kernel_stats.csv"
    ;;
  shardbudget)
    # per-rank kernel costs of the pixel-sharded C4 solve at N = 2, 4, 8 (bench.py --shard1
    # --shard-of N: rank 0's shard on a one-rank RCCL communicator), kernel trace + stats each.
    # gram_err_min=0: the error monitor keeps the Gram form on every iteration, as the global
    # solve does (the shard's own problem would otherwise fall back to the explicit x-forming
    # reconstruction, which runs on the step stream on a communicator)
    # (SHARD_RANK: which rank's shard; rank 0's shard of the 8-way cut is all background, x_true = 0,
    # so its own error monitor cannot take the Gram form; the global solve's does)
    for nn in ${@:-2 4 8}; do
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/shard_of$nn" -o trace \
          -- python3 bench.py --workload c4 --shard1 --shard-of $nn --shard-rank $(( ${SHARD_RANK:-0} % nn )) \
             --steps 5 --warmup 1 --no-cpu-baseline --opt gram_err_min=0 \
          > "$O/shard_of$nn.log" 2>&1 || { tail -20 "$O/shard_of$nn.log"; exit 1; }
      bench_line "$O/shard_of$nn.log" > "$O/${TAG}_bench_c4_shard_of$nn.json"
      cp "$(find "$O/shard_of$nn" -name '*kernel_stats.csv' | head -1)" "$O/${TAG}_c4_shard_of${nn}_kernel_stats.csv"
      cp "$(find "$O/shard_of$nn" -name '*kernel_trace.csv' | head -1)" "$O/c4_shard_of${nn}_kernel_trace.csv"
    done
    ;;
  tests)
    n=$(ls "$O"/${TAG}_gpu_tests_*.log 2>/dev/null | wc -l)
    timeout -k 10 1200 python -u -m pytest -m gpu -v --timeout 400 --timeout-method thread "$@" \
        > "$O/${TAG}_gpu_tests_$n.log" 2>&1
    rc=$?
    tail -3 "$O/${TAG}_gpu_tests_$n.log"
    exit $rc
    ;;
  bench)
    wl=$1; shift
    timeout -k 10 600 python -u bench.py --workload "$wl" "$@" > "$O/bench_$wl.log" 2>&1 || { tail -20 "$O/bench_$wl.log"; exit 1; }
    bench_line "$O/bench_$wl.log" | tee "$O/${TAG}_bench_$wl.json"
    ;;
  trace)
    wl=$1; shift
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$wl" -o trace \
        -- python3 bench.py --workload "$wl" --steps 5 --warmup 1 --no-cpu-baseline "$@" > "$O/trace_$wl.log" 2>&1 || exit 1
    bench_line "$O/trace_$wl.log" > "$O/${TAG}_bench_${wl}_traced.json"
    cp "$(find "$O/trace_$wl" -name '*kernel_stats.csv' | head -1)" "$O/${TAG}_${wl}_kernel_stats.csv"
    head -12 "$O/${TAG}_${wl}_kernel_stats.csv"
    ;;
  traffic)
    wl=$1; shift
    nm=${NAME:-$wl}
    B="bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline --no-timing $*"
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$O/pmc_$nm/$c" -o p \
          -- python3 $B > "$O/pmc_${nm}_$c.log" 2>&1 || { tail -5 "$O/pmc_${nm}_$c.log"; exit 1; }
    done
    python3 scripts/summarize_profile.py --traffic "$O/pmc_$nm" "$nm" > "$O/traffic_$nm.json" || exit 1
    cat "$O/traffic_$nm.json"
    ;;
  pmc)
    wl=$1; shift
    B="bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline --no-timing"
    i=0
    for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
               "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS" \
               "FETCH_SIZE" "WRITE_SIZE"; do
      i=$((i + 1))
      timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$O/pmc_$wl/p$i" -o p$i \
          -- python3 $B > "$O/pmc_${wl}_p$i.log" 2>&1 || { tail -5 "$O/pmc_${wl}_p$i.log"; exit 1; }
    done
    python3 scripts/pmc_fused_summary.py "$O/pmc_$wl" "$O/pmc_$wl/summary.json" && cat "$O/pmc_$wl/summary.json"
    ;;
  micro)
    f=f64; [ "${F32:-0}" = 1 ] && f=f32
    HGM_MICRO_F32=${F32:-0} timeout -k 10 600 python -u scripts/fused_micro.py "$@" > "$O/${TAG}_micro_$f.jsonl" 2>&1 || exit 1
    grep variant "$O/${TAG}_micro_$f.jsonl"
    ;;
  ab)
    rounds=$1; shift
    : > "$O/${TAG}_ab.jsonl"
    for r in $(seq "$rounds"); do
      side=0
      for args in "$@"; do
        side=$((side + 1))
        timeout -k 10 600 python -u bench.py $args > "$O/ab.log" 2>&1 || { tail -20 "$O/ab.log"; exit 1; }
        python3 -c "
import json, sys
d = json.loads([l for l in open('$O/ab.log') if l.startswith('{')][-1])
print(json.dumps({'round': $r, 'side': $side, 'args': '''$args''', 'value': d['value'],
                  'kernels': {k: round(v['avg_us'], 2) for k, v in d['kernels'].items()}}))" | tee -a "$O/${TAG}_ab.jsonl"
      done
    done
    ;;
  libab)
    old=$1; shift
    : > "$O/${TAG}_lib_ab.jsonl"
    for wl in "$@"; do
      for rep in 1 2; do
        HGM_LIB=$old timeout -k 10 300 python -u scripts/time_ops.py "$wl" >> "$O/${TAG}_lib_ab.jsonl" 2>> "$O/lib_ab.err" || exit 1
        timeout -k 10 300 python -u scripts/time_ops.py "$wl" >> "$O/${TAG}_lib_ab.jsonl" 2>> "$O/lib_ab.err" || exit 1
      done
    done
    cat "$O/${TAG}_lib_ab.jsonl"
    ;;
  *)
    sed -n 2,28p "$0"
    exit 2
    ;;
esac
