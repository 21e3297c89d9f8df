"""Entry order inside the rows of the tiled ray-major A: Siddon traversal order (as generated)
against ascending stored column (the device transpose of the transpose), per workload."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT, os.path.join(ROOT, "scripts")]
import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402
from shard_kernels import time_spmv  # noqa: E402


def main():
    lib = L.load()
    ctx = hgmres.Context(0)
    for N, na, dt in ((2048, 19, L.HGM_F64), (4096, 47, L.HGM_F32), (4096, 47, L.HGM_F64)):
        A = hgmres.SparseOperator.siddon(N, na, ctx=ctx, dtype=dt)
        B = A.T
        S = B.T
        for rep in range(2):
            ra = time_spmv(ctx, lib, A, 20)
            rs = time_spmv(ctx, lib, S, 20)
            print(N, na, "f32" if dt == L.HGM_F32 else "f64", "traversal", round(ra[0], 4), "sorted", round(rs[0], 4),
                  flush=True)
        for M in (A, B, S):
            M.close()


if __name__ == "__main__":
    main()
