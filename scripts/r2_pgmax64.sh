#!/bin/bash
# LDS page budget per chunk, fp64 at C4: 256 / 320 / 384 pages.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/lib_sweep.jsonl
bash scripts/lib_sweep.sh c4 exp/lib_base.so exp/lib_p64_320.so exp/lib_p64_384.so || exit $?
