"""Strip width with the dual strips: isolated A product at 32/64/128-pixel strips (two alternating
rounds).  usage: python scripts/band_sweep_dual.py c3|c4|c5"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT, os.path.join(ROOT, "scripts")]
import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402
import bench  # noqa: E402
from shard_kernels import time_spmv  # noqa: E402


def main():
    w = sys.argv[1]
    wl = bench.WORKLOADS[w]
    lib = L.load()
    ctx = hgmres.Context(0)
    dt = L.HGM_F32 if wl.get("f32") else L.HGM_F64
    A = hgmres.SparseOperator.siddon(wl["N"], wl["angles"], ctx=ctx, dtype=dt)
    N = wl["N"]
    for rep in range(2):
        for s in (32, 64, 128):
            A.set_bands(s * N)
            r = time_spmv(ctx, lib, A, 20)
            print(json.dumps({"wl": w, "strip": s, "rep": rep, "A_ms": round(r[0], 4)}), flush=True)


if __name__ == "__main__":
    main()
