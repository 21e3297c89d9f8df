"""SpMV kernel sweep on device-generated tomography operators.

For each config and operator (A: ray-major, long rows; B = A': pixel-major, short
rows) times (band width, lanes, variant) choices with HIP events on the library
stream; one JSON line per case with algorithmic GB/s =
(nnz*(s+4) + 8*(rows+1) + s*cols + s*rows) / average launch time.
usage: python scripts/spmv_sweep.py [c2 c3 c4] [--reps 20] [--quick]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]

import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402
from hgmres.problems import CONFIGS  # noqa: E402


def time_case(ctx, lib, M, xd, yd, reps):
    for _ in range(3):
        lib.hgm_spmv(ctx.handle, M._h, xd, yd)
    ctx.kernel_timing(True)
    for _ in range(reps):
        lib.hgm_spmv(ctx.handle, M._h, xd, yd)
    ms, calls, by = ctx.kernel_timing_read(0)
    ctx.kernel_timing(False)
    avg = ms / calls
    return avg * 1e3, by / calls / (avg / 1e3) / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c2", "c3", "c4"])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--tiles", default="1", help="comma list of stored pixel orders tile[:super_block]")
    ap.add_argument("--cases", default="", help="comma list band_w:band_group:group:variant (only --ops)")
    ap.add_argument("--ops", default="A", help="operators the --cases apply to (A, B or AB)")
    a = ap.parse_args()
    lib = L.load()
    ctx = hgmres.Context(0)
    for cfg, tile in [(c, t) for c in a.configs for t in a.tiles.split(",")]:
        tt, _, ss = tile.partition(":")
        sup = int(ss or 0)
        N, na = CONFIGS[cfg]
        t0 = time.time()
        A = hgmres.SparseOperator.siddon(N, na, ctx=ctx, order=(int(tt), sup))
        B = A.T
        ctx.synchronize()
        gen_s = time.time() - t0
        for name, M in (("A", A), ("B", B)):
            rows, cols = M.shape
            xd, yd = C.c_void_p(), C.c_void_p()
            lib.hgm_dev_alloc(ctx.handle, 8 * cols, C.byref(xd))
            lib.hgm_dev_alloc(ctx.handle, 8 * rows, C.byref(yd))
            ones = np.ones(cols)
            lib.hgm_memcpy_h2d(ctx.handle, xd, ones.ctypes.data_as(C.c_void_p), 8 * cols)
            # (band_width, band_group, group (rows kernel) or stream-reduction lanes, variant)
            if a.cases and name in a.ops:
                cases = [tuple(int(v) for v in cs.split(":")) for cs in a.cases.split(",")]
            elif a.cases:
                continue
            elif name == "A" and a.quick and sup:
                cases = [(0, 0, 32, 1)]
                for w in (sup * sup, 2 * sup * sup, 4 * sup * sup):
                    if w < cols:
                        cases += [(w, 8, 32, 8), (w, 8, 16, 8), (w, 16, 0, 1)]
            elif name == "A" and a.quick:
                cases = [(0, 0, 32, 1), (0, 0, 64, 1), (0, 0, 32, 8)]
                cases += [(w, 8, 32, 8) for w in (1 << 17, 1 << 19, 1 << 21) if w < cols]
            elif name == "A":
                widths = [0] + ([w for w in (1 << 17, 1 << 18, 1 << 19, 1 << 20) if w < cols])
                cases = []
                for w in widths:
                    if w == 0:
                        cases += [(0, 0, 32, 1), (0, 0, 32, 3), (0, 0, 32, 8), (0, 0, 64, 8), (0, 0, 64, 10)]
                    else:
                        cases += [(w, 8, 0, 1), (w, 8, 8, 8), (w, 8, 16, 8), (w, 8, 32, 8), (w, 8, 16, 10)]
            elif a.quick:
                cases = [(0, 0, 8, 0), (0, 0, 4, 8), (0, 0, 8, 8)]
            else:
                cases = [(0, 0, 8, 0), (0, 0, 8, 1), (0, 0, 4, 8), (0, 0, 8, 8), (0, 0, 16, 8), (0, 0, 8, 10)]
            cur_w = None
            for (w, bg, g, v) in cases:
                if w != cur_w:
                    M.set_bands(w, bg)
                    cur_w = w
                elif w:
                    M.set_bands(w, bg)
                M.tune(v, g if g else 0)
                us, gbs = time_case(ctx, lib, M, xd, yd, a.reps)
                print(json.dumps({"cfg": cfg, "tile": tile, "op": name, "rows": rows, "cols": cols, "nnz": M.nnz,
                                  "band_w": w, "band_group": bg, "group": g, "variant": v,
                                  "avg_us": round(us, 2), "GBps": round(gbs, 1), "gen_s": round(gen_s, 2)}),
                      flush=True)
            lib.hgm_dev_free(ctx.handle, xd)
            lib.hgm_dev_free(ctx.handle, yd)
        A.close()
        B.close()
    ctx.close()


if __name__ == "__main__":
    main()
