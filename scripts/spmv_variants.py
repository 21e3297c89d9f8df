"""Time the A and B SpMV kernels of a config under several kernel choices (hgm_mat_tune
variant:group; give the creation default explicitly, e.g. C2 A 1:16, B 0:8), HIP events on the library stream,
alternating the choices `rounds` times.  Prints per-choice averages and whether each choice's
product is bitwise the auto one.
usage: python scripts/spmv_variants.py c2 reps rounds A=1:16,26:4,24:8 B=0:8,26:4
(v:g:band_width:band_group also re-bands the operator first)"""
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
    cfg, reps, rounds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    choices = dict(a.split("=", 1) for a in sys.argv[4:])
    lib = L.load()
    ctx = hgmres.Context(0)
    N, na = CONFIGS[cfg]
    f32 = os.environ.get("HGM_DTYPE") == "f32"
    es = 4 if f32 else 8
    A = hgmres.SparseOperator.siddon(N, na, ctx=ctx, dtype=L.HGM_F32 if f32 else L.HGM_F64)
    B = A.T
    res = {"cfg": cfg}
    for nm, M in (("A", A), ("B", B)):
        if nm not in choices:
            continue
        rows, cols = M.shape
        xd, yd = C.c_void_p(), C.c_void_p()
        lib.hgm_dev_alloc(ctx.handle, es * cols, C.byref(xd))
        lib.hgm_dev_alloc(ctx.handle, es * rows, C.byref(yd))
        xs = np.random.default_rng(0).standard_normal(cols).astype(np.float32 if f32 else np.float64)
        lib.hgm_memcpy_h2d(ctx.handle, xd, xs.ctypes.data_as(C.c_void_p), es * cols)
        opts = choices[nm].split(",")
        acc = {o: [] for o in opts}
        ys = {}
        for r in range(rounds):
            for o in opts:
                parts = [int(t) for t in o.split(":")]
                if len(parts) >= 4:                      # v:g:band_width:band_group
                    M.set_bands(parts[2], parts[3])
                M.tune(parts[0], parts[1])
                for _ in range(3):
                    lib.hgm_spmv(ctx.handle, M._h, xd, yd)
                ctx.kernel_timing(True)
                for _ in range(reps):
                    lib.hgm_spmv(ctx.handle, M._h, xd, yd)
                ms, calls, by = ctx.kernel_timing_read(0)
                ctx.kernel_timing(False)
                acc[o].append(ms / calls)
                y = np.empty(rows, dtype=xs.dtype)
                lib.hgm_memcpy_d2h(ctx.handle, y.ctypes.data_as(C.c_void_p), yd, es * rows)
                ys[o] = y
                res.setdefault("bytes_" + nm, by / calls)
        base = ys[opts[0]]
        for o in opts:
            avg = float(np.mean(acc[o]))
            res[f"{nm}_{o}"] = {"avg_us": round(avg * 1e3, 2), "runs_us": [round(t * 1e3, 2) for t in acc[o]],
                                "GBps_alg": round(res["bytes_" + nm] / avg / 1e6, 1),
                                "bitwise_vs_first": bool(np.array_equal(ys[o], base)),
                                "maxrel_vs_first": float(np.max(np.abs(ys[o] - base)) / np.max(np.abs(base)))}
            print(nm, o, res[f"{nm}_{o}"], flush=True)
        lib.hgm_dev_free(ctx.handle, xd)
        lib.hgm_dev_free(ctx.handle, yd)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
