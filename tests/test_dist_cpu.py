"""Multi-rank DECOMPOSITION on the CPU (no GPU), world_size 2 over torch.distributed gloo.

What this checks is the arithmetic of the pixel sharding of DESIGN.md §5, re-derived in numpy:
it does NOT call libhgmres (no GPU here; the library's own multi-rank code runs on the GPU box
in tests/test_gpu_parity.py::test_shard_emulation_two_ranks and, at full size as 2, 4 and 8 ranks,
tests/test_gpu_fullsize.py::test_c4_c5_sharded_vs_oracle).
* the shard plan and the shard operators (hgmres.dist) are exact slices whose partial
  products sum to the full ones;
* a sharded BA-RTP GMRES written in numpy with the library's exchange pattern (one all-reduce of
  the m-vector partial A_g q_g per operator application, one scalar all-reduce per MGS inner
  product, nothing else) reproduces the single-process oracle (oracle/restatement.py,
  hybrid_ba_gmres_rtp.m) to 1e-10.
"""
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden_problem
from hgmres.dist import plan_pixel_shards, shard_operators
from oracle import restatement as R


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_plan_pixel_shards_cover_and_balance(world):
    A, B, b, xt, g = golden_problem("tomo24_matched.npz")
    plan = plan_pixel_shards(A, world, B)
    n = A.shape[1]
    assert plan[0][0] == 0 and plan[-1][1] == n
    assert all(plan[i][1] == plan[i + 1][0] for i in range(world - 1))
    w = np.diff(sp.csc_matrix(A).indptr) + np.diff(sp.csr_matrix(B).indptr)
    loads = [w[lo:hi].sum() for lo, hi in plan]
    assert max(loads) - min(loads) <= 2 * w.max() + 1     # balanced to within a pixel's nnz


def test_shard_operators_are_exact_slices():
    A, B, b, xt, g = golden_problem("tomo24_matched.npz")
    rng = np.random.default_rng(0)
    x = rng.standard_normal(A.shape[1])
    y = rng.standard_normal(A.shape[0])
    parts = []
    for lo, hi in plan_pixel_shards(A, 3, B):
        Ag, Bg = shard_operators(A, B, lo, hi)
        assert Ag.shape == (A.shape[0], hi - lo) and Bg.shape == (hi - lo, A.shape[0])
        parts.append(Ag @ x[lo:hi])
        np.testing.assert_allclose(Bg @ y, (B @ y)[lo:hi], rtol=0, atol=1e-12)
    np.testing.assert_allclose(sum(parts), A @ x, rtol=1e-13, atol=1e-12)


def _sharded_ba_rtp(rank, world, port, maxit, lam, out):
    """BA-RTP GMRES (hybrid_ba_gmres_rtp.m:3-40) on this rank's pixel shard."""
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allsum(v):
        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64))
        dist.all_reduce(t)
        return t.numpy()

    A, B, b, xt, g = golden_problem("tomo24_matched.npz")
    lo, hi = plan_pixel_shards(A, world, B)[rank]
    Ag, Bg = shard_operators(A, B, lo, hi)
    M = lambda q: Bg @ allsum(Ag @ q) + lam * q                       # noqa: E731  :6 M_reg_op
    dot = lambda a, c: float(allsum(np.array([a @ c]))[0])            # noqa: E731  n-space inner product
    r0 = Bg @ b                                                        # :7-9 (B*b - M_reg(0))
    beta = np.sqrt(dot(r0, r0))
    Q = np.zeros((hi - lo, maxit + 1))
    H = np.zeros((maxit + 1, maxit))
    Q[:, 0] = r0 / beta
    xs = []
    for k in range(maxit):
        v = M(Q[:, k])                                                 # :19
        for j in range(k + 1):                                         # :20-23 MGS
            H[j, k] = dot(Q[:, j], v)
            v = v - H[j, k] * Q[:, j]
        H[k + 1, k] = np.sqrt(dot(v, v))                               # :24
        if H[k + 1, k] == 0:
            break
        Q[:, k + 1] = v / H[k + 1, k]
        rhs = np.zeros(k + 2)
        rhs[0] = beta
        y = R.mldivide(H[: k + 2, : k + 1], rhs)                       # :28-29
        xs.append(Q[:, : k + 1] @ y)                                   # :30
    out[rank] = {"lo": lo, "hi": hi, "H": H, "x": xs[-1]}
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_two_rank_sharded_gmres_matches_oracle():
    import torch.multiprocessing as mp
    world, maxit, lam = 2, 8, 1e-2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_sharded_ba_rtp, args=(world, _free_port(), maxit, lam, out), nprocs=world, join=True)
    A, B, b, xt, g = golden_problem("tomo24_matched.npz")
    xr, er, rr, kr, Hr = R.hybrid_ba_gmres_rtp(A, B, b, xt, 0.0, maxit, lam, return_H=True)
    x = np.zeros(A.shape[1])
    for r in range(world):
        x[out[r]["lo"]:out[r]["hi"]] = out[r]["x"]
        # every rank holds the same (replicated) Hessenberg matrix
        np.testing.assert_allclose(out[r]["H"], Hr, rtol=0, atol=1e-10 * np.abs(Hr).max())
    assert np.linalg.norm(x - xr) <= 1e-10 * np.linalg.norm(xr)


def test_stored_pixel_index_is_the_tiled_permutation():
    """hgmres.core.stored_pixel_index mirrors csrc/ops.hip pixel_index: a permutation; 4 x 4
    tiles in tile-column-major order, column-major inside a tile; super-blocks contiguous."""
    from hgmres.core import stored_pixel_index
    N = 8
    s = stored_pixel_index(N, 4, 0)
    assert sorted(s.tolist()) == list(range(N * N))
    assert s[1 + 5 * N] == ((1 * 2 + 0) * 4 + 1) * 4 + 1      # (r=1, c=5): tile (0,1), (col 1, row 1) inside
    assert list(s[:4]) == [0, 1, 2, 3] and s[N] == 4            # first tile column-major
    t = stored_pixel_index(16, 4, 8)
    assert sorted(t.tolist()) == list(range(256))
    assert t[0 + 8 * 16] == 2 * 64                              # (r=0, c=8): third super-block (column-major)
    np.testing.assert_array_equal(stored_pixel_index(8, 1, 0), np.arange(64))


@pytest.mark.parametrize("N,tile", [(64, 4), (256, 4), (128, 1)])
def test_dual_strip_band_key_is_the_pixel_strip(N, tile):
    """The band key of the dual strips (csrc/ops.hip BandKey) restated on the host:
    in the tile-column-major stored order, s / (64 N) is the 64-pixel COLUMN strip and
    (s mod tile*N) / (64 tile) the 64-pixel ROW strip of the pixel; the coordinates row_steep
    recovers from s are the pixel's own; and a shard window of whole tile columns keeps both
    keys, with row strips of h = W N / cols rows (the column strips' pixel count)."""
    from hgmres.core import stored_pixel_index
    p = np.arange(N * N, dtype=np.int64)
    r, c = p % N, p // N
    s = stored_pixel_index(N, tile, 0)
    W, t, Nt = 64 * N if N >= 128 else 16 * N, tile, N // tile
    h = W // N
    np.testing.assert_array_equal(s // W, c // h)
    np.testing.assert_array_equal((s % (t * N)) // (h * t), r // h)
    q = s // (t * t)
    np.testing.assert_array_equal((q % Nt) * t + s % t, r)          # pixel row from s
    np.testing.assert_array_equal((q // Nt) * t + (s // t) % t, c)  # pixel column from s
    # a shard of tile columns [4, 4 + k): local stored positions s - lo
    k = N // (2 * t)
    lo, hi = 4 * t * N, (4 + k) * t * N
    sel = (s >= lo) & (s < hi)
    sl = s[sel] - lo
    cols = hi - lo
    hs = W * N // cols
    assert hs % t == 0 and N % hs == 0
    np.testing.assert_array_equal((sl % (t * N)) // (hs * t), r[sel] // hs)
    assert N // hs == -(-cols // W)            # as many row strips as column strips
