# MGS one-reduction tile width (HGM_OPT_MGS1_PPL: pairs per lane; 0 = by length, 2 at m = 272k) on
# the m-space basis of the N = 8 shard (rank 3), HIP-event MGS time per step
set -o pipefail
O=gpurun_out/r6; mkdir -p $O; : > $O/r6_mgs_ppl_shard8.jsonl
for r in 1 2; do
  for ppl in 0 1 4; do
    timeout -k 10 300 python -u bench.py --workload c4 --shard1 --shard-of 8 --shard-rank 3 --steps 10 --warmup 2 \
        --no-cpu-baseline --time-classes MGS --time-every 1 --opt mgs1_ppl=$ppl > $O/mgsppl.log 2>&1 || { tail -5 $O/mgsppl.log; exit 1; }
    python3 -c "
import json
d = json.loads([l for l in open('$O/mgsppl.log') if l.startswith('{')][-1])
print(json.dumps({'round': $r, 'mgs1_ppl': $ppl, 'value': d['value'], 'kernels': {k: round(v['avg_us'], 2) for k, v in d['kernels'].items()}}))" | tee -a $O/r6_mgs_ppl_shard8.jsonl
  done
done
