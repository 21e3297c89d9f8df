"""Multi-GPU plumbing: pixel sharding and communicator set-up.

Partitioning: the pixel dimension n is cut into ``world`` contiguous ranges
balanced by the nnz each rank streams per Krylov step (``nnz(A(:,P_g)) +
nnz(B(P_g,:))``).  Rank g owns ``A_g = A(:,P_g)`` (ray-major CSR with local
column indices) and ``B_g = B(P_g,:)``; n-vectors are sharded, m-vectors
replicated, and the only data-path collective is the sum of the m-vector
partials ``A_g q_g`` (one RCCL all-reduce per operator application) plus scalar
all-reduces for n-space inner products — done inside libhgmres.

Communicators: one process per GPU.  :func:`init_context` creates an RCCL
communicator from a unique id broadcast over an existing ``torch.distributed``
group (gloo or nccl); :func:`host_allreduce_context` routes the same sums
through a ``torch.distributed`` CPU group instead (shard emulation: several
processes on ONE device, used by the tests).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import scipy.sparse as sp

from . import _lib as L
from .core import Context, HgmError


def plan_pixel_shards(A, world: int, B=None):
    """Contiguous pixel ranges [(lo, hi), ...] balancing nnz(A(:,P)) + nnz(B(P,:))."""
    n = A.shape[1]
    if world < 1:
        raise ValueError("world must be >= 1")
    Ac = sp.csc_matrix(A)
    w = np.diff(Ac.indptr).astype(np.float64)
    if B is not None:
        w = w + np.diff(sp.csr_matrix(B).indptr).astype(np.float64)
    cum = np.concatenate([[0.0], np.cumsum(w)])
    total = cum[-1]
    bounds = [0]
    for g in range(1, world):
        target = total * g / world
        j = int(np.searchsorted(cum, target, side="left"))
        j = max(bounds[-1], min(j, n))
        bounds.append(j)
    bounds.append(n)
    return [(bounds[g], bounds[g + 1]) for g in range(world)]


def tile_column_shards(N: int, world: int, tile: int):
    """Pixel shards of a device-generated N x N operator in its tiled STORED order: `world`
    contiguous ranges [(lo, hi), ...] of stored positions made of whole tile columns (tile * N
    stored pixels each), as equal as the tile-column count allows.  Parallel-beam nnz per
    pixel is uniform, so equal pixel counts balance nnz (0.02 % at 8 shards, checked at 512^2);
    every shard keeps the tiled gather locality and the 64-column bands of the single-GPU
    kernels (bench.py build_shard)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    n = N * N
    col = max(tile, 1) * N
    ncol = n // col
    if world > ncol:
        raise ValueError(f"{world} shards of {ncol} tile columns")
    bounds = [0] + [int(round(g * ncol / world)) * col for g in range(1, world)] + [n]
    return [(bounds[g], bounds[g + 1]) for g in range(world)]


def shard_operators(A, B, lo: int, hi: int):
    """(A_g, B_g) for the pixel range [lo, hi): A(:,lo:hi) as CSR with local
    columns, B(lo:hi,:) as CSR."""
    A_g = sp.csc_matrix(A)[:, lo:hi].tocsr()
    B_g = sp.csr_matrix(B)[lo:hi, :].tocsr()
    return A_g, B_g


def unique_id() -> bytes:
    buf = (C.c_char * L.HGM_UNIQUE_ID_BYTES)()
    rc = L.load().hgm_comm_unique_id(buf)
    if rc != L.HGM_OK:
        raise HgmError(f"hgm_comm_unique_id failed ({rc})")
    return bytes(buf)


def init_context(device: int, rank: int, world: int, uid: bytes | None = None, group=None,
                 one_rank_comm: bool = False) -> Context:
    """RCCL-backed context.  If ``uid`` is None it is created on rank 0 and
    broadcast with ``torch.distributed.broadcast_object_list`` over ``group``.
    ``one_rank_comm`` (world 1): a one-rank communicator, so the solve runs the sharded
    code path with real RCCL all-reduces on one GPU."""
    if world == 1 and one_rank_comm and uid is None:
        uid = unique_id()
    if world > 1 and uid is None:
        import torch.distributed as dist
        obj = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        uid = obj[0]
    if uid is None:
        uid = bytes(L.HGM_UNIQUE_ID_BYTES)
    buf = (C.c_char * L.HGM_UNIQUE_ID_BYTES).from_buffer_copy(uid)
    h = C.c_void_p()
    rc = L.load().hgm_ctx_create_dist(device, rank, world, buf, C.byref(h))
    if rc != L.HGM_OK:
        raise HgmError(f"hgm_ctx_create_dist(rank={rank}, world={world}) failed ({rc})")
    return Context(device, _handle=h)


def host_allreduce_context(device: int, rank: int, world: int, group=None) -> Context:
    """Context whose cross-rank sums go through torch.distributed (CPU tensors)."""
    import torch
    import torch.distributed as dist
    ctx = Context(device)

    def _sum(arr: np.ndarray):
        t = torch.from_numpy(arr)          # shares memory with the staging buffer
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)

    ctx.set_host_allreduce(rank, world, _sum)
    return ctx
