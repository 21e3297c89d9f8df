"""Experiment: does the pixel (column) order of A change the SpMV time?

The ray-major A gathers x at the pixels a ray crosses.  In the reference's column-major
pixel order a ray walking along j jumps N pixels (one cache line per entry); in a tiled
order (T x T pixel tiles, tile-major) consecutive crossings share lines.  This times
hgm_spmv on A(:, perm) and on its transpose for several orders (same nnz, same values).
usage: python scripts/pixel_order_bench.py [cfg] [--reps 50]
"""
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


def tile_perm(N, T):
    """new index -> old column-major pixel index, T x T tiles in tile-major order."""
    i, j = np.meshgrid(np.arange(N), np.arange(N), indexing="ij")   # pixel (i, j), old = i + j*N
    ti, tj = i // T, j // T
    key = ((tj * (N // T) + ti) * T + (j % T)) * T + (i % T)
    old = (i + j * N).ravel()
    order = np.argsort(key.ravel(), kind="stable")
    return old[order]


def morton_perm(N):
    i, j = np.meshgrid(np.arange(N), np.arange(N), indexing="ij")
    def spread(v):
        v = v.astype(np.uint64)
        out = np.zeros_like(v)
        for b in range(16):
            out |= ((v >> np.uint64(b)) & np.uint64(1)) << np.uint64(2 * b)
        return out
    key = spread(i.ravel()) | (spread(j.ravel()) << np.uint64(1))
    old = (i + j * N).ravel()
    return old[np.argsort(key, kind="stable")]


def timed(ctx, lib, M, reps):
    rows, cols = M.shape
    xd, yd = C.c_void_p(), C.c_void_p()
    lib.hgm_dev_alloc(ctx.handle, 8 * cols, C.byref(xd))
    lib.hgm_dev_alloc(ctx.handle, 8 * rows, C.byref(yd))
    ones = np.ones(cols)
    lib.hgm_memcpy_h2d(ctx.handle, xd, ones.ctypes.data_as(C.c_void_p), 8 * cols)
    for _ in range(3):
        lib.hgm_spmv(ctx.handle, M._h, xd, yd)
    ctx.kernel_timing(True)
    for _ in range(reps):
        lib.hgm_spmv(ctx.handle, M._h, xd, yd)
    ms = 0.0
    calls = 0
    for cls in (0, 1):
        t, n_, _ = ctx.kernel_timing_read(cls)
        ms += t
        calls += n_
    ctx.kernel_timing(False)
    lib.hgm_dev_free(ctx.handle, xd)
    lib.hgm_dev_free(ctx.handle, yd)
    return ms / max(calls, 1) * 1e3


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cfg = args[0] if args else "c2"
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 50
    lib = L.load()
    ctx = hgmres.Context(0)
    N, na = CONFIGS[cfg]
    A0 = hgmres.SparseOperator.siddon(N, na, ctx=ctx, order="reference").to_scipy().tocsc()
    orders = {"colmajor": np.arange(N * N)}
    for T in (2, 4, 8, 16):
        orders[f"tile{T}"] = tile_perm(N, T)
    orders["morton"] = morton_perm(N)
    for name, perm in orders.items():
        Ap = A0[:, perm].tocsr()
        Ap.sort_indices()
        A = hgmres.SparseOperator.from_scipy(Ap, ctx)
        B = A.T
        ta = timed(ctx, lib, A, reps)
        tb = timed(ctx, lib, B, reps)
        print(json.dumps({"cfg": cfg, "order": name, "A_us": round(ta, 2), "B_us": round(tb, 2),
                          "A_variant": A.variant if hasattr(A, "variant") else None}), flush=True)
        del A, B
    ctx.close()


if __name__ == "__main__":
    main()
