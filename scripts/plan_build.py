"""One-pass plan build at a BASELINE geometry: the device build (HGM_OPT_FUSED_PLAN_DEV = 1) against
the host build (= 0) on the same operator -- seconds, partial slots, and whether the two plans are
byte-identical (checksum).  usage: python scripts/plan_build.py [N angles [f32]]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
import torch  # noqa: E402,F401
import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402

N, na = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (4096, 47)))
f32 = len(sys.argv) > 3 and sys.argv[3] == "f32"
ctx = hgmres.Context(0)
A = hgmres.SparseOperator.siddon(N, na, ctx=ctx, dtype=L.HGM_F32 if f32 else L.HGM_F64)
B = A.T
ctx.synchronize()
out = {"N": N, "angles": na, "dtype": "f32" if f32 else "f64", "nnz": A.nnz}
for dev in (1, 0, 1):
    with ctx.options(fused_plan_dev=dev):
        t0 = time.perf_counter()
        info = hgmres.fused_plan_info(A, B)
        out[f"{'device' if dev else 'host'}_build"] = dict(info, wall_s=round(time.perf_counter() - t0, 3))
print(json.dumps(out))
