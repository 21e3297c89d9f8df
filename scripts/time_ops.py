"""Time the workload's A and B = A' products (HIP events on the library stream), for A/B
comparisons of library builds (HGM_LIB=<path> selects the build).
usage: python scripts/time_ops.py c3|c4|c5 [reps]"""
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
    wl = bench.WORKLOADS[sys.argv[1]]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    lib = L.load()
    ctx = hgmres.Context(0)
    dt = L.HGM_F32 if wl.get("f32") else L.HGM_F64
    A = hgmres.SparseOperator.siddon(wl["N"], wl["angles"], ctx=ctx, dtype=dt)
    B = A.T
    out = {"lib": os.environ.get("HGM_LIB", "default"), "wl": sys.argv[1]}
    for rep in range(2):
        ra = time_spmv(ctx, lib, A, reps)
        rb = time_spmv(ctx, lib, B, reps)
        out[f"A{rep}"], out[f"B{rep}"] = round(ra[0], 4), round(rb[0], 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
