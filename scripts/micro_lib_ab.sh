#!/bin/bash
# Alternating hgm_spmv_ab micro runs of two library builds (HGM_LIB=OLD.so vs the in-tree build),
# ROUNDS rounds, fp64 and fp32: bash scripts/micro_lib_ab.sh OLD.so ROUNDS VARIANT
# -> gpurun_out/$TAG/micro_lib_ab.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${TAG:-r5}
O=gpurun_out/$TAG
mkdir -p "$O"
old=$1; rounds=${2:-3}; var=${3:-w4r32q4}
: > "$O/micro_lib_ab.txt"
for f in 0 1; do
  for i in $(seq "$rounds"); do
    HGM_LIB=$old HGM_MICRO_F32=$f timeout -k 10 200 python -u scripts/fused_micro.py 4096 47 50 two,$var > "$O/m.log" 2>&1 || { tail "$O/m.log"; exit 1; }
    grep variant "$O/m.log" | sed "s/^/old /" | tee -a "$O/micro_lib_ab.txt"
    HGM_MICRO_F32=$f timeout -k 10 200 python -u scripts/fused_micro.py 4096 47 50 two,$var > "$O/m.log" 2>&1 || { tail "$O/m.log"; exit 1; }
    grep variant "$O/m.log" | sed "s/^/new /" | tee -a "$O/micro_lib_ab.txt"
  done
done
