#!/bin/bash
# C2 env A/B sweep (under gpurun): MGS partial granularity and pipeline depth.
cd "$GRAFT_REPO_ROOT"
V=$' | \nHGM_MGS1_PPL=1 | \nHGM_MGS1_PPL=4 | \nHGM_MGS_PPL=2 | \nHGM_PIPE_DEPTH=1 | \nHGM_PIPE_DEPTH=3 | \n | \nHGM_MGS1_PPL=1 | \nHGM_MGS_PPL=2 | '
VARIANTS="$V" bash scripts/ab_bench.sh
