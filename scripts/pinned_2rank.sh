#!/bin/bash
# ADVICE r4 (host spins): the 2-rank pixel-sharded solve (both ranks on GPU 0, host all-reduce
# hook) with both ranks pinned to two cores, host waits spinning-then-yielding
# (HGM_OPT_HOST_SPIN_US = 200) against the blocking waits (-1) and the default (auto: -1 on
# fewer than 4 cores), alternating.
# -> gpurun_out/$TAG/pinned_2rank.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${TAG:-r5}
O=gpurun_out/$TAG
mkdir -p "$O"
: > "$O/pinned_2rank.jsonl"
for r in 1 2; do
  for spin in 200 -1 auto; do
    opt="--opt host_spin_us=$spin"; [ $spin = auto ] && opt=
    timeout -k 10 300 taskset -c 0,1 python -u bench.py --gpus 2 --same-device --comm host --workload c3 \
        --steps 3 --warmup 1 --no-cpu-baseline $opt > "$O/pinned.log" 2>&1 || { tail -20 "$O/pinned.log"; exit 1; }
    python3 -c "
import json
d = json.loads([l for l in open('$O/pinned.log') if l.startswith('{')][-1])
print(json.dumps({'round': $r, 'host_spin_us': '$spin', 'cores': '0,1', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" | tee -a "$O/pinned_2rank.jsonl"
  done
done
