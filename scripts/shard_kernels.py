"""Per-rank SpMV cost of the sharded C4 solve, measured on one GPU: build rank 0's tiled
stored-order shard for world = 2, 4, 8 exactly as bench.py does (build_shard) and time its
A_g and B_g products (HIP events on the library stream).  Rank 0's shard is representative:
parallel-beam nnz per pixel is uniform, so the shards are balanced to 0.02 %.
usage: python scripts/shard_kernels.py [reps] [dual modes, e.g. 0,1,2: A re-banded under each
HGM_OPT_BAND_DUAL value]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402
import bench  # noqa: E402


def time_spmv(ctx, lib, M, reps):
    rows, cols = M.shape
    xd, yd = C.c_void_p(), C.c_void_p()
    lib.hgm_dev_alloc(ctx.handle, 8 * cols, C.byref(xd))
    lib.hgm_dev_alloc(ctx.handle, 8 * rows, C.byref(yd))
    xs = np.random.default_rng(0).standard_normal(cols)
    lib.hgm_memcpy_h2d(ctx.handle, xd, xs.ctypes.data_as(C.c_void_p), 8 * cols)
    for _ in range(3):
        lib.hgm_spmv(ctx.handle, M._h, xd, yd)
    ctx.kernel_timing(True)
    for _ in range(reps):
        lib.hgm_spmv(ctx.handle, M._h, xd, yd)
    ms, calls, by = ctx.kernel_timing_read(0)
    ctx.kernel_timing(False)
    lib.hgm_dev_free(ctx.handle, xd)
    lib.hgm_dev_free(ctx.handle, yd)
    return ms / calls, by / calls


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    modes = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [None]
    lib = L.load()
    ctx = hgmres.Context(0)
    wl = bench.WORKLOADS["c4"]
    out = {}
    for world in (1, 2, 4, 8):
        if world == 1:
            A = hgmres.SparseOperator.siddon(wl["N"], wl["angles"], ctx=ctx)
            B = A.T
        else:
            A, B, b, xs, (lo, hi), full = bench.build_shard(ctx, wl, 0, world)
        rb = time_spmv(ctx, lib, B, reps)
        for mode in modes:
            if mode is not None:
                ctx.set_option("band_dual", float(mode))
                A.set_bands(64 * wl["N"])
            ra = time_spmv(ctx, lib, A, reps)
            key = world if mode is None else f"{world}/dual{mode}"
            out[key] = {"A_ms": round(ra[0], 4), "A_GBps": round(ra[1] / ra[0] / 1e6, 1), "A_nnz": A.nnz,
                        "B_ms": round(rb[0], 4), "B_GBps": round(rb[1] / rb[0] / 1e6, 1)}
            print(key, out[key], flush=True)
        A.close()
        B.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
