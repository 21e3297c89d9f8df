"""Time the C4 (or C3) A and B SpMV kernels with and without paged x gathers (variant bit 16),
HIP events on the library stream (hgm_kernel_timing).  Bitwise check between the two.
usage: python scripts/spmv_ab.py [c4|c3] [reps] [f32]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402
from hgmres.problems import CONFIGS  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dt = L.HGM_F32 if "f32" in sys.argv else L.HGM_F64
    es = 4 if dt == L.HGM_F32 else 8
    lib = L.load()
    ctx = hgmres.Context(0)
    N, na = CONFIGS[cfg]
    A = hgmres.SparseOperator.siddon(N, na, ctx=ctx, dtype=dt)
    B = A.T
    res = {"cfg": cfg, "dtype": "f32" if es == 4 else "f64"}
    for nm, M in (("A", A), ("B", B)):
        rows, cols = M.shape
        xd, yd = C.c_void_p(), C.c_void_p()
        lib.hgm_dev_alloc(ctx.handle, es * cols, C.byref(xd))
        lib.hgm_dev_alloc(ctx.handle, es * rows, C.byref(yd))
        xs = np.random.default_rng(0).standard_normal(cols).astype(np.float32 if es == 4 else np.float64)
        lib.hgm_memcpy_h2d(ctx.handle, xd, xs.ctypes.data_as(C.c_void_p), es * cols)
        ys = {}
        for v in (8 | 2, 8 | 2 | 16):
            M.tune(v, 4)
            for _ in range(3):
                lib.hgm_spmv(ctx.handle, M._h, xd, yd)
            ctx.kernel_timing(True)
            for _ in range(reps):
                lib.hgm_spmv(ctx.handle, M._h, xd, yd)
            ms, calls, by = ctx.kernel_timing_read(0)
            ctx.kernel_timing(False)
            y = np.empty(rows, dtype=xs.dtype)
            lib.hgm_memcpy_d2h(ctx.handle, y.ctypes.data_as(C.c_void_p), yd, es * rows)
            ys[v] = y
            avg = ms / calls
            res[f"{nm}_v{v}"] = {"avg_ms": round(avg, 4), "GBps_alg": round(by / calls / avg / 1e6, 1)}
            print(nm, v, res[f"{nm}_v{v}"], flush=True)
        res[f"{nm}_bitwise"] = bool(np.array_equal(ys[10], ys[26]))
        print(nm, "bitwise", res[f"{nm}_bitwise"], flush=True)
        lib.hgm_dev_free(ctx.handle, xd)
        lib.hgm_dev_free(ctx.handle, yd)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
