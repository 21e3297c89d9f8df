#!/bin/bash
# C3 MGS sweep variants (under gpurun): Krylov column padding (HGM_OPT_KRYLOV_PAD) with the
# library as built.  Per variant: the bench line, and the per-step dots/update durations from a
# kernel trace (scripts/mgs_steps.py).  VARIANTS="name:pad ..." (default: pad 0 vs auto).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/mgsab
mkdir -p $O
for v in ${VARIANTS:-p0:0 auto:-1 p0b:0 autob:-1}; do
  name=${v%%:*}; pad=${v##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$name -o t \
      -- python3 bench.py --workload c3 --steps 4 --warmup 1 --no-cpu-baseline --opt krylov_pad=$pad > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
  echo "$name $(grep -o '"value": [0-9.]*' $O/$name.log | head -1)"
  python3 scripts/mgs_steps.py $(find $O/$name -name '*kernel_trace.csv' | head -1) 4194304 20 | tail -1
done
