# one collective per Golub-Kahan iteration on a communicator (ridden monitor partials) vs the
# previous library (separate scalar all-reduces): C5 LSQR / LSMR on a one-rank RCCL communicator
# (--shard1) and on rank 3's shard of an 8-way cut, alternating builds
set -o pipefail
O=gpurun_out/r6; mkdir -p $O; : > $O/r6_ride_ab.jsonl
PREV=$PWD/hybrid-gmres_amd/hgmres/libhgmres_prev.so
for r in 1 2; do
  for wl in c5 c5m; do
    for lib in prev new; do
      if [ $lib = prev ]; then export HGM_LIB=$PREV; else unset HGM_LIB; fi
      for cut in 1 8; do
        timeout -k 10 300 python -u bench.py --workload $wl --shard1 --shard-of $cut --shard-rank $((3 % cut)) --steps 10 --warmup 2 \
            --no-cpu-baseline --no-timing > $O/ride.log 2>&1 || { tail -5 $O/ride.log; exit 1; }
        python3 -c "
import json
d = json.loads([l for l in open('$O/ride.log') if l.startswith('{')][-1])
print(json.dumps({'round': $r, 'wl': '$wl', 'lib': '$lib', 'shard_of': $cut, 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" | tee -a $O/r6_ride_ab.jsonl
      done
    done
  done
done
