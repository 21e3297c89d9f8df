set -o pipefail
O=gpurun_out/r6
mkdir -p $O
: > $O/r6_mgs_ab.jsonl
for r in 1 2; do
  for lib in default mgs16; do
    if [ $lib = mgs16 ]; then export HGM_LIB=$PWD/hybrid-gmres_amd/hgmres/libhgmres_mgs16.so; else unset HGM_LIB; fi
    timeout -k 10 300 python -u bench.py --workload c4 --shard1 --shard-of 8 --shard-rank 3 --steps 10 --warmup 2 --no-cpu-baseline --time-classes ALL --time-every 1 > $O/mgsab.log 2>&1 || { tail -20 $O/mgsab.log; exit 1; }
    python3 -c "
import json
d = json.loads([l for l in open('$O/mgsab.log') if l.startswith('{')][-1])
print(json.dumps({'round': $r, 'lib': '$lib', 'value': d['value'], 'kernels': {k: round(v['avg_us'], 2) for k, v in d['kernels'].items()}}))" | tee -a $O/r6_mgs_ab.jsonl
  done
done
unset HGM_LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_parity.py::test_shard_emulation_two_ranks -k "res_img or shard_emulation or dbg or reduce_by_band or failed_plan or rowpair or not_taken" -s > $O/r6_t4.log 2>&1; grep -E "lsqr res img|passed|failed|FAILED" $O/r6_t4.log | tail -12
