"""Why the shard A_g streams slower than the generated A: time the C4 A as generated
(Siddon traversal order inside each row), as a device transpose of its transpose (rows sorted
by stored column), and as bench.py's one-rank shard (row_slice of A', transposed)."""
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
    N, na = 4096, 47
    A = hgmres.SparseOperator.siddon(N, na, ctx=ctx)
    r = time_spmv(ctx, lib, A, 10)
    print("generated", round(r[0], 4), round(r[1] / r[0] / 1e6, 1), flush=True)
    B = A.T
    A.close()
    A2 = B.T
    r = time_spmv(ctx, lib, A2, 10)
    print("transpose^2 (auto bands)", round(r[0], 4), round(r[1] / r[0] / 1e6, 1), flush=True)
    A2.close()
    S = B.row_slice(0, B.shape[0])
    B.close()
    A3 = S.T
    r = time_spmv(ctx, lib, A3, 10)
    print("shard1 auto bands", round(r[0], 4), round(r[1] / r[0] / 1e6, 1), flush=True)
    A3.set_bands(64 * N, 0)
    r = time_spmv(ctx, lib, A3, 10)
    print("shard1 64N bands", round(r[0], 4), round(r[1] / r[0] / 1e6, 1), flush=True)


if __name__ == "__main__":
    main()
