#!/bin/bash
# k_fused_reduce variants (lanes per ray, HGM_FUSED_RG build define): kernel-trace stats of the
# C4 one-pass micro-benchmark with each library (under gpurun).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for r in 1 2; do
  for L in hybrid-gmres_amd/hgmres/libhgmres.so exp/libhgmres_rg1.so exp/libhgmres_rg16.so; do
    t=$(basename $L .so)_$r
    HGM_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rd/$t -o s \
        -- python3 scripts/fused_micro.py 4096 47 20 f1024 > gpurun_out/rd/$t.log 2>&1 || exit 1
    echo "$t $(grep '^{' gpurun_out/rd/$t.log | cut -c1-80) $(grep -h 'fused' $(find gpurun_out/rd/$t -name '*kernel_stats.csv') | awk -F'",' '{split($2,a,","); print substr($1,1,28), a[3]}' | tr '\n' ' ')"
  done
done
