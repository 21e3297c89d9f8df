# partial-reduction lanes per ray on 8-way shards (experiments build: fused_reduce 2/3/4 = 1/2/4 lanes)
set -o pipefail
export HGM_LIB=$PWD/hybrid-gmres_amd/hgmres/libhgmres_exp.so
O=gpurun_out/r6; mkdir -p $O; : > $O/r6_reduce_lanes_shard8.jsonl
for r in 1 2; do
  for red in 0 2 3 4; do
    timeout -k 10 300 python -u scripts/shard_balance.py 8 30 - fused_reduce=$red 0,3 2>/dev/null | grep opts | tee -a $O/r6_reduce_lanes_shard8.jsonl || exit 1
  done
done
