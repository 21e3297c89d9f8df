# one-pass region side on 8-way shards (rank 3) and on the full C4 operator (world 1)
set -o pipefail
O=gpurun_out/r6; mkdir -p $O; : > $O/r6_region_shard8.jsonl
for r in 1 2; do
  for reg in 32 24 28 20 16; do
    timeout -k 10 300 python -u scripts/shard_balance.py 8 30 - fused_wregion=$reg 3 2>/dev/null | grep opts | tee -a $O/r6_region_shard8.jsonl || exit 1
  done
done
for reg in 32 24; do
  timeout -k 10 300 python -u scripts/shard_balance.py 1 10 - fused_wregion=$reg 2>/dev/null | grep opts | tee -a $O/r6_region_shard8.jsonl || exit 1
done
