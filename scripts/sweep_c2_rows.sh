cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
true || timeout -k 10 600 python scripts/spmv_sweep.py c2 --tiles 4 --ops A --cases "0:0:8:1,0:0:16:1,0:0:32:1,0:0:64:1,0:0:16:3,0:0:32:3,0:0:16:5,0:0:32:5,0:0:16:0,0:0:32:0,0:0:64:0" > gpurun_out/swA.log 2>&1 || exit 1
timeout -k 10 600 python scripts/spmv_sweep.py c2 --tiles 4 --ops B --cases "0:0:4:1,0:0:8:1,0:0:16:1,0:0:4:0,0:0:8:0,0:0:4:3,0:0:8:3,0:0:4:5,0:0:8:5" > gpurun_out/swB.log 2>&1 || exit 1
grep -h "^{" gpurun_out/swB.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['op'], 'g', d['group'], 'v', d['variant'], 'bw', d['band_w'], d['avg_us'], d['GBps'])"
