#!/bin/bash
# C2 A SpMV traffic attribution (scripts/c2_stream_split.py): per mode (real / zero columns / the
# bench's tiled operator) one rocprofv3 --pmc run per counter group.  Output under gpurun_out/$TAG/c2split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r5}
O=gpurun_out/$TAG/c2split
mkdir -p "$O"
timeout -k 10 60 rocprofv3 --list-avail > "$O/list_avail.txt" 2>&1 || true
for mode in real zero tiled; do
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCP_TCC_READ_REQ_sum TCC_REQ_sum"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$O/$mode/p$i" -o p \
        -- python3 scripts/c2_stream_split.py $mode 50 > "$O/${mode}_p$i.log" 2>&1 || { echo "pass $mode $grp failed"; tail -3 "$O/${mode}_p$i.log"; }
  done
done
for mode in real zero tiled; do echo "### $mode"; python3 scripts/pmc_kernels.py "$O/$mode"; done > "$O/summary.txt" 2>&1
grep -A12 "k_spmv" "$O/summary.txt" | head -80
