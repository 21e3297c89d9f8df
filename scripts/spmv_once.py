"""Run a few SpMV launches per (operator, variant, group) — the target of rocprofv3
PMC passes (FETCH_SIZE / WRITE_SIZE / TCC_HIT / TCC_MISS) in scripts/profile_spmv.sh.
Prints the launch order so counter rows can be matched to cases.
usage: python scripts/spmv_once.py CFG [A:v:g[:band_w:band_group] ...] [--reps 3]
(stored pixel order of the generated operator: env HGM_SIDDON_TILE / HGM_SIDDON_SUPER;
 HGM_DTYPE=f32 for the fp32 operator)
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]

import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402
from hgmres.problems import CONFIGS  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    reps = 3
    if "--reps" in sys.argv:
        reps = int(sys.argv[sys.argv.index("--reps") + 1])
        args = [a for a in args if a != str(reps)]
    cfg, cases = args[0], args[1:] or ["A:1:32", "B:1:8"]
    lib = L.load()
    ctx = hgmres.Context(0)
    N, na = CONFIGS[cfg]
    order = (int(os.environ.get("HGM_SIDDON_TILE", "1")), int(os.environ.get("HGM_SIDDON_SUPER", "0")))
    f32 = os.environ.get("HGM_DTYPE") == "f32"
    es = 4 if f32 else 8
    A = hgmres.SparseOperator.siddon(N, na, ctx=ctx, order=order, dtype=L.HGM_F32 if f32 else L.HGM_F64)
    B = A.T
    ops = {"A": A, "B": B}
    bufs = {}
    for nm, M in ops.items():
        rows, cols = M.shape
        xd, yd = C.c_void_p(), C.c_void_p()
        lib.hgm_dev_alloc(ctx.handle, es * cols, C.byref(xd))
        lib.hgm_dev_alloc(ctx.handle, es * rows, C.byref(yd))
        ones = np.ones(cols, dtype=np.float32 if f32 else np.float64)
        lib.hgm_memcpy_h2d(ctx.handle, xd, ones.ctypes.data_as(C.c_void_p), es * cols)
        bufs[nm] = (xd, yd)
    for case in cases:
        parts = case.split(":")
        nm, v, g = parts[:3]
        M = ops[nm]
        if len(parts) >= 5:                      # A:variant:group:band_width:band_group
            M.set_bands(int(parts[3]), int(parts[4]))
        M.tune(int(v), int(g))
        xd, yd = bufs[nm]
        for _ in range(reps):
            lib.hgm_spmv(ctx.handle, M._h, xd, yd)
        ctx.synchronize()
        print(f"case {cfg} {case} rows={M.shape[0]} cols={M.shape[1]} nnz={M.nnz} launches={reps}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
