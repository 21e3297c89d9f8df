#!/bin/bash
# fp32 page staging at C5: one round (exp/lib_base.so), rounds in a loop (exp/lib_loop.so),
# one-round fast path + loop (in-tree build).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/lib_sweep.jsonl
bash scripts/lib_sweep.sh c5 exp/lib_base.so exp/lib_loop.so hybrid-gmres_amd/hgmres/libhgmres.so || exit $?
