"""Isolated SpMV throughput vs operator size (default kernel choice, auto pixel order):
does a working set that fits the 256 MB MALL stream faster than one that does not?
usage: python scripts/spmv_size_scan.py [angles] [N ...]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402


def main():
    na = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    Ns = [int(v) for v in sys.argv[2:]] or [181, 256, 362, 512, 724, 1024]
    lib = L.load()
    ctx = hgmres.Context(0)
    for N in Ns:
        A = hgmres.SparseOperator.siddon(N, na, ctx=ctx)
        B = A.T
        for name, M in (("A", A), ("B", B)):
            rows, cols = M.shape
            xd, yd = C.c_void_p(), C.c_void_p()
            lib.hgm_dev_alloc(ctx.handle, 8 * cols, C.byref(xd))
            lib.hgm_dev_alloc(ctx.handle, 8 * rows, C.byref(yd))
            ones = np.ones(cols)
            lib.hgm_memcpy_h2d(ctx.handle, xd, ones.ctypes.data_as(C.c_void_p), 8 * cols)
            for _ in range(5):
                lib.hgm_spmv(ctx.handle, M._h, xd, yd)
            ctx.kernel_timing(True)
            for _ in range(50):
                lib.hgm_spmv(ctx.handle, M._h, xd, yd)
            ms, calls, by = ctx.kernel_timing_read(0)
            ctx.kernel_timing(False)
            us = ms / calls * 1e3
            print(json.dumps({"N": N, "angles": na, "op": name, "nnz": M.nnz, "MB": round(by / calls / 1e6, 1),
                              "avg_us": round(us, 2), "GBps": round(by / calls / (us * 1e-6) / 1e9, 1)}), flush=True)
            lib.hgm_dev_free(ctx.handle, xd)
            lib.hgm_dev_free(ctx.handle, yd)
        A.close()
        B.close()
    ctx.close()


if __name__ == "__main__":
    main()
