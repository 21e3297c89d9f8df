# k_fused_reduce duration per library build (rocprofv3 kernel trace of the micro-benchmark):
#   bash scripts/reduce_libab.sh LIB1.so LIB2.so ...  (F32=1 for fp32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r4}/reduce_ab; mkdir -p $O
i=0
for r in 1 2; do
  for lib in "$@"; do
    i=$((i + 1))
    export HGM_LIB=$lib HGM_MICRO_F32=${F32:-0}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$i -o t -- python3 scripts/fused_micro.py 4096 47 20 w4r32 > $O/t$i.log 2>&1 || exit 1
    python3 - "$lib" $(find $O/t$i -name '*kernel_stats.csv' | head -1) <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[2])):
    if 'k_fused' in r['Name']:
        print(sys.argv[1], r['Name'].split('(')[0][-40:], r['Calls'], round(float(r['AverageNs']) / 1e3, 2))
PY
  done
done
