# Alternating bench lines of two libraries on one box: HGM_LIB=OLD.so against the in-tree library,
# per workload, ROUNDS rounds.  -> gpurun_out/libab${AB_TAG}/lib_ab_bench.jsonl
# usage: bash scripts/lib_ab_bench.sh OLD.so ROUNDS WL [WL ...]   (a WL may carry bench args: "c4 --shard1 ...")
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/libab${AB_TAG:-}; mkdir -p $O
old=$1; rounds=$2; shift 2
: > $O/lib_ab_bench.jsonl
for r in $(seq "$rounds"); do
  for wl in "$@"; do
    for side in old new; do
      if [ $side = old ]; then
        HGM_LIB=$old timeout -k 10 400 python -u bench.py --no-cpu-baseline --workload $wl > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
      else
        timeout -k 10 400 python -u bench.py --no-cpu-baseline --workload $wl > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
      fi
      python3 -c "
import json
d = json.loads([l for l in open('$O/ab.log') if l.startswith('{')][-1])
print(json.dumps({'round': $r, 'workload': '''$wl''', 'side': '$side', 'value': d['value'], 'ms_per_step': d['ms_per_step'],
                  'kernels': {k: round(v['avg_us'], 2) for k, v in d['kernels'].items()}}))" | tee -a $O/lib_ab_bench.jsonl
    done
  done
done
