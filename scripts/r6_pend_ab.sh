# Round 6: the one pass's staging (batched branch-free loads, run table and first row pointers in
# flight with the q gathers) and the opt-in m-space pending normalisation (pend_norm=2: the one pass
# stages q = v / h; no k_mgs_normalize) A/B.  Alternating bench lines, one box: the previous library
# (HGM_LIB=$1), the new library (default), the new library with pend_norm=2, at N = 1 (C4), on rank
# 3's shard of the 8-way cut (one-rank RCCL, bench.py --shard1) and at C5 (the fp32 pass).
# usage: bash scripts/r6_pend_ab.sh OLD.so [ROUNDS]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6pend${AB_TAG:-}; mkdir -p $O
old=$1
rounds=${2:-2}
: > $O/r6_pend_ab.jsonl
SH="--workload c4 --shard1 --shard-of 8 --shard-rank 3 --opt gram_err_min=0"
one() {   # label, lib ('' = new), bench args
  local label=$1 lib=$2; shift 2
  if [ -n "$lib" ]; then
    HGM_LIB=$lib timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  else
    timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  fi
  python3 -c "
import json
d = json.loads([l for l in open('$O/ab.log') if l.startswith('{')][-1])
print(json.dumps({'round': $r, 'side': '$label', 'value': d['value'], 'ms_per_step': d['ms_per_step'],
                  'kernels': {k: round(v['avg_us'], 2) for k, v in d['kernels'].items()}}))" | tee -a $O/r6_pend_ab.jsonl
}
for r in $(seq $rounds); do
  one old_n1 "$old" || exit 1
  one new_n1 "" || exit 1
  one pend2_n1 "" --opt pend_norm=2 || exit 1
  one old_shard8 "$old" $SH || exit 1
  one new_shard8 "" $SH || exit 1
  one pend2_shard8 "" $SH --opt pend_norm=2 || exit 1
  one old_c5 "$old" --workload c5 || exit 1
  one new_c5 "" --workload c5 || exit 1
done
