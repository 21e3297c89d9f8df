"""The RCCL transport on one GPU: a one-rank communicator (hgm_ctx_create_dist with world 1 and
a real unique id) sends every solver down the sharded code path of SURVEY.md §8(e) with real
ncclAllReduce calls on the m-vector partials and the n-space scalars.  With one rank the sums
are identities, so each solve must reproduce the single-context solve of the same operator.
A multi-rank RCCL run needs one GPU per rank (RCCL refuses two ranks on one device); the
2-rank host-hook emulation in test_gpu_parity.py covers the cross-rank arithmetic."""
import os
import sys

import numpy as np
import pytest

import hgmres
from hgmres.dist import init_context

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _shard_worker import solve_all  # noqa: E402

pytestmark = pytest.mark.gpu

TOL = 1e-10


def rel(a, b):
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-300)


def test_one_rank_rccl_matches_single_context():
    ctx1 = init_context(0, 0, 1, one_rank_comm=True)
    try:
        r = solve_all(ctx1, 0, 1)
    finally:
        ctx1.close()
    ctx0 = hgmres.Context(0)
    try:
        s = solve_all(ctx0, 0, 1)
    finally:
        ctx0.close()
    tols = {"hba": TOL, "abp": TOL, "abn": TOL, "abnd": TOL, "hab": TOL, "tabn": TOL, "thba": TOL,
            "lsqr": 1e-7, "lsqr32": 1e-4,          # the Golub-Kahan envelope of the shard test
            "tlsqr32": 1e-4, "tlsmr32": 1e-4}      # (fp32 one-pass shards; the same code path at one rank)
    for tag, tol in tols.items():
        assert rel(r[f"{tag}_x"], s[f"{tag}_x"]) < tol, tag
        assert rel(r[f"{tag}_res"], s[f"{tag}_res"]) < tol, tag
        assert rel(r[f"{tag}_err"], s[f"{tag}_err"]) < tol, tag
    # (the GCV minimum is flat: lambda itself is ill-determined at 1e-4, the minimum value is not)
    assert rel(r["gcv_H"], s["gcv_H"]) < TOL and abs(r["gcv_val"] - s["gcv_val"]) <= 1e-10 * s["gcv_val"]
    for tag in ("hba", "abn", "hab", "tabn", "thba"):
        assert r[f"{tag}_H"].shape == s[f"{tag}_H"].shape
        assert rel(r[f"{tag}_H"], s[f"{tag}_H"]) < TOL, tag


def test_one_rank_rccl_gcv():
    """hgm_gcv_function on the BA side all-reduces n over the communicator (capi gcv)."""
    from hgmres.problems import tomo_problem
    P = tomo_problem(32, 45, noise=1e-2, seed=1)
    ctx1 = init_context(0, 0, 1, one_rank_comm=True)
    ctx0 = hgmres.Context(0)
    try:
        for side in ("ab", "ba"):
            g1 = hgmres.gcv_function(1e-2, P.A, P.B, P.b, P.A.shape[0], 8, side, ctx=ctx1)
            g0 = hgmres.gcv_function(1e-2, P.A, P.B, P.b, P.A.shape[0], 8, side, ctx=ctx0)
            assert abs(g1 - g0) <= TOL * abs(g0), side
    finally:
        ctx1.close()
        ctx0.close()
