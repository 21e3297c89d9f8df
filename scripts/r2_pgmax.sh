#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for P in 256 320 384; do
  if [ $P = 256 ]; then L=hybrid-gmres_amd/hgmres/libhgmres.so; else L=hybrid-gmres_amd/hgmres/libhgmres_pg$P.so; fi
  HGM_LIB=$L timeout -k 10 300 python -u scripts/spmv_ab.py c4 20 > gpurun_out/pgmax_$P.log 2>&1 || exit $?
done
HGM_LIB=hybrid-gmres_amd/hgmres/libhgmres.so timeout -k 10 300 python -u scripts/spmv_ab.py c4 20 > gpurun_out/pgmax_256b.log 2>&1 || exit $?
