#!/bin/bash
# Alternating A/B of the library as built against exp/libhgmres_old.so (under gpurun):
# isolated A/B products (scripts/time_ops.py) and bench lines, per workload in WLS.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for wl in ${WLS:-c3 c4}; do
  for r in 1 2; do
    for lib in exp/libhgmres_old.so hybrid-gmres_amd/hgmres/libhgmres.so; do
      tag=$(basename $lib .so)
      echo "$wl $tag $(HGM_LIB=$lib timeout -k 10 300 python scripts/time_ops.py $wl 20 2>/dev/null | grep '^{')"
    done
  done
done
for wl in ${BWLS:-c3}; do
  for r in 1 2; do
    for lib in exp/libhgmres_old.so hybrid-gmres_amd/hgmres/libhgmres.so; do
      tag=$(basename $lib .so)
      v=$(HGM_LIB=$lib timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --time-classes AB 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})")
      echo "bench $wl $tag $v"
    done
  done
done
