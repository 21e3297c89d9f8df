cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for r in 1 2; do for L in hybrid-gmres_amd/hgmres/libhgmres.so exp/libhgmres_a2.so; do
  for wl in c3 c5; do
    v=$(HGM_LIB=$L timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --time-classes AB 2>/dev/null | grep '^{' | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], {k: round(v['avg_us'],1) for k,v in d['kernels'].items()})")
    echo "$wl $(basename $L) $v"
  done
  echo "c4iso $(basename $L) $(HGM_LIB=$L timeout -k 10 300 python scripts/time_ops.py c4 10 2>/dev/null | grep '^{')"
done; done
