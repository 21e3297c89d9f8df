#!/bin/bash
# C2 bench under SpMV variant overrides (variant:group; 1 VEC, 2 NT, 4 XCD).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for ta in "" "1:16" "3:32" "5:32" "0:32"; do
for tb in "" "2:8" "4:8"; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline ${ta:+--tune-a $ta} ${tb:+--tune-b $tb} > gpurun_out/t.log 2>&1 || exit 1
  echo "A[$ta] B[$tb] $(grep -o '"value": [0-9.]*' gpurun_out/t.log | head -1) $(grep -o '"avg_launch_us": [0-9.]*' gpurun_out/t.log)"
done
done
