set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4
bash scripts/gpu.sh evidence || exit 1
for wl in c2 c3 c3gcv c5 c5m; do
  bash scripts/gpu.sh bench $wl --no-cpu-baseline || exit 1
done
