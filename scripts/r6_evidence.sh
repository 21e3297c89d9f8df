# Round-6 evidence on one MI355X (gpurun): part A = the GPU suite + smoke, part B = bench lines
# (default C4 with cpu_baseline, its rocprofv3 kernel trace, the side workloads with cpu_baseline).
# usage: [TAG=name] bash scripts/r6_evidence.sh A|B   (outputs gpurun_out/$TAG/$TAG_*; default r6final)
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r6final}
O=gpurun_out/$T; mkdir -p $O
bench_line() { grep '^{' "$1" | tail -1; }
case "$1" in
  A)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s -rA --timeout 900 --timeout-method thread \
        > $O/${T}_gpu_tests.log 2>&1 || { grep -E "passed|failed" $O/${T}_gpu_tests.log | tail -3; exit 1; }
    grep -E "passed|failed" $O/${T}_gpu_tests.log | tail -2
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.txt 2>&1 || exit 1
    cat $O/${T}_smoke.txt | grep smoke
    ;;
  B)
    timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
    bench_line $O/bench_default.log > $O/${T}_bench_default_c4.json; cat $O/${T}_bench_default_c4.json | cut -c1-300
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_default -o trace \
        -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/trace_default.log 2>&1 || exit 1
    bench_line $O/trace_default.log > $O/${T}_bench_default_c4_traced.json
    cp "$(find $O/trace_default -name '*kernel_stats.csv' | head -1)" $O/${T}_default_kernel_stats.csv
    for wl in c2 c3 c3gcv c5 c5m; do
      timeout -k 10 600 python -u bench.py --workload $wl > $O/bench_$wl.log 2>&1 || { tail -20 $O/bench_$wl.log; exit 1; }
      bench_line $O/bench_$wl.log > $O/${T}_bench_$wl.json; cut -c1-200 $O/${T}_bench_$wl.json
    done
    ;;
esac
