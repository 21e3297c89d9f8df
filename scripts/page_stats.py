"""Pages of x touched per streaming chunk (4096 entries) of the C3/C4 SpMV operators: sizes
the LDS x-page staging of the paged streaming kernel.  Host-only analysis.
usage: python scripts/page_stats.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
from hgmres.problems import siddon_projector  # noqa: E402

CH = 4096


def tiled_index(N, tile=4):
    """stored index of reference pixel p = col*N + row (4x4 tiles, tile-column-major)."""
    p = np.arange(N * N)
    col, row = p // N, p % N
    tc, tr = col // tile, row // tile
    return ((tc * (N // tile) + tr) * tile * tile + (col % tile) * tile + (row % tile)).astype(np.int64)


def chunk_pages(ci, page):
    nch = (ci.size + CH - 1) // CH
    pad = np.full(nch * CH - ci.size, -1)
    pg = np.concatenate([ci // page, pad]).reshape(nch, CH)
    s = np.sort(pg, axis=1)
    return ((s[:, 1:] != s[:, :-1]) & (s[:, 1:] >= 0)).sum(axis=1) + (s[:, 0] >= 0)


def report(tag, ci):
    for page in (16, 32):
        c = chunk_pages(ci, page)
        print(f"{tag:28s} page {page * 8:4d} B: pages/chunk mean {c.mean():6.1f}  p50 {np.median(c):5.0f}  "
              f"p99 {np.percentile(c, 99):5.0f}  max {c.max():5d}  LDS(max) {c.max() * page * 8 / 1024:6.1f} KiB")


def main():
    # B = A' (pixel-major rows, ray columns): local structure does not depend on N much
    N, na = 1024, 47
    A = siddon_projector(N, na).tocsr()
    st = tiled_index(N)
    At = A.tocsc()                                  # columns = pixels (reference order)
    Bt = A.T.tocsr()                                # rows = pixels (reference order)
    order = np.argsort(st)                          # stored row order (tiled)
    Bs = Bt[order]
    report(f"B N={N} {na} angles (tiled)", Bs.indices.astype(np.int64))
    # A (ray-major) at the C4 width, a few angles, banded in 256Ki-pixel bands of the tiled order
    N, na = 4096, 5
    A = siddon_projector(N, na).tocsr()
    st = tiled_index(N)
    col = st[A.indices]
    W = 1 << 18
    band = col // W
    rows = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    key = band * A.shape[0] + rows                   # band-major, then row, entries in ray order
    o = np.argsort(key, kind="stable")
    report(f"A N={N} banded 256Ki (tiled)", col[o])
    del At


if __name__ == "__main__":
    main()
