set -o pipefail
cd "$GRAFT_REPO_ROOT" && export TMPDIR=/tmp && O=gpurun_out/r4/gap && mkdir -p $O
run() {  # name, extra bench args
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$1 -o t -- python3 bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline $2 > $O/$1.log 2>&1 || return 1
  echo "== $1"; grep '^{' $O/$1.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])"
  python3 scripts/trace_gaps.py $(find $O/$1 -name '*kernel_trace.csv' | head -1) 300
}
run base "" && run notiming "--no-timing" && HIP_FORCE_DEV_KERNARG=1 run devkarg "--no-timing" && run nopend "--no-timing --opt pend_norm=0" && run nopoll "--no-timing --opt ring_poll=0"
