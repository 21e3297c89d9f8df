"""Degenerate inputs through the C ABI, against the oracle's MATLAB semantics: the reference has
no input validation, so these pin what MATLAB's arithmetic does (NaN from 0/0, Inf from x/0,
breakdown at k = 1 leaving x unassigned) and that the device path neither hangs on such values
(the pinned-ring sentinel is a NaN no kernel produces) nor raises where MATLAB would not."""
import warnings

import numpy as np
import pytest
import scipy.sparse as sp

import hgmres
from hgmres.problems import tomo_problem
from oracle import restatement as R

pytestmark = pytest.mark.gpu


def _same(a, b):
    """Equal as MATLAB would print them: NaN where NaN, Inf where Inf, else within 1e-10."""
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape
    assert np.array_equal(np.isnan(a), np.isnan(b))
    fin = np.isfinite(b)
    assert np.array_equal(np.isinf(a), np.isinf(b))
    if fin.any():
        assert np.max(np.abs(a[fin] - b[fin])) <= 1e-10 * max(np.max(np.abs(b[fin])), 1e-300)


@pytest.fixture(scope="module")
def P():
    return tomo_problem(24, 12, noise=1e-2, seed=0)


def _oracle(fn, *args):
    with warnings.catch_warnings(), np.errstate(all="ignore"):
        warnings.simplefilter("ignore")
        return fn(*args)


@pytest.mark.parametrize("name", ["hybrid_ba_gmres_rtp", "lsqr_solver", "lsmr_solver"])
def test_zero_rhs_gives_matlabs_nans(gpu_ctx, P, name):
    """b = 0: beta = 0 and the first normalisation is 0/0 (hybrid_ba_gmres_rtp.m:10-13,
    lsqr_solver.m:7-8): NaN histories and x, exactly where MATLAB has them; no hang."""
    b = np.zeros(P.A.shape[0])
    args = {"hybrid_ba_gmres_rtp": (P.A, P.B, b, P.x_true, 0.0, 4, 1e-2),
            "lsqr_solver": (P.A, b, P.x_true, 0.0, 4),
            "lsmr_solver": (P.A, b, P.x_true, 0.0, 4)}[name]
    g = getattr(hgmres, name)(*args, ctx=gpu_ctx)
    r = _oracle(getattr(R, name), *args)
    assert g[-1] == r[-1]                      # niters
    for a, b_ in zip(g[:-1], r[:-1]):
        _same(a, b_)


def test_zero_x_true_gives_inf_error(gpu_ctx, P):
    """x_true = 0: error_norm = norm(x - 0)/0 = Inf (hybrid_ab_gmres_rtp.m:36)."""
    xt = np.zeros(P.A.shape[1])
    g = hgmres.hybrid_ab_gmres_rtp(P.A, P.B, P.b, xt, 0.0, 5, 1e-2, ctx=gpu_ctx)
    r = _oracle(R.hybrid_ab_gmres_rtp, P.A, P.B, P.b, xt, 0.0, 5, 1e-2)
    assert np.all(np.isinf(g[1])) and g[3] == r[3]
    _same(g[0], r[0])
    _same(g[2], r[2])


def test_one_by_one_system(gpu_ctx):
    """n = m = 1: the Krylov space is exhausted after one step (H(2,1) = 0, the break of
    hybrid_ba_gmres_rtp.m:25), with x assigned from the zero initial guess (:4)."""
    A = sp.csr_matrix(np.array([[2.0]]))
    B = sp.csr_matrix(np.array([[0.5]]))
    b, xt = np.array([3.0]), np.array([3.0])
    g = hgmres.hybrid_ba_gmres_rtp(A, B, b, xt, 0.0, 3, 0.0, ctx=gpu_ctx)
    r = _oracle(R.hybrid_ba_gmres_rtp, A, B, b, xt, 0.0, 3, 0.0)
    assert g[3] == r[3] == 1
    for a, b_ in zip(g[:3], r[:3]):
        _same(a, b_)
    with pytest.raises(hgmres.OutputNotAssigned):      # AB-RTP never assigns x on that break
        hgmres.hybrid_ab_gmres_rtp(A, B, b, xt, 0.0, 3, 0.0, ctx=gpu_ctx)
    with pytest.raises(R.OutputNotAssigned):
        R.hybrid_ab_gmres_rtp(A, B, b, xt, 0.0, 3, 0.0)


def test_maxit_one_everywhere(gpu_ctx, P):
    """maxit = 1 for every solver: one iteration, histories of length 1."""
    for name, args in (("hybrid_ab_gmres_rtp", (P.A, P.B, P.b, P.x_true, 0.0, 1, 1e-2)),
                       ("hybrid_ba_gmres_rtp", (P.A, P.B, P.b, P.x_true, 0.0, 1, 1e-2)),
                       ("ABgmres_nonhybrid_bounds", (P.A, P.B, P.b, P.x_true, 0.0, 1)),
                       ("BAgmres_hybrid_bounds", (P.A, P.B, P.b, P.x_true, 0.0, 1, 1e-2)),
                       ("lsqr_solver", (P.A, P.b, P.x_true, 0.0, 1)),
                       ("lsmr_solver", (P.A, P.b, P.x_true, 0.0, 1)),
                       ("hybrid_lsqr_solver", (P.A, P.b, P.x_true, 0.0, 1, 1e-2)),
                       ("hybrid_lsmr_solver", (P.A, P.b, P.x_true, 0.0, 1, 1e-2))):
        g = getattr(hgmres, name)(*args, ctx=gpu_ctx)
        r = _oracle(getattr(R, name), *args)
        k = 4 if name == "lsmr_solver" else 3
        assert g[k] == r[k] == 1, name
        for a, b_ in zip(g[:k], r[:k]):
            _same(a, b_)


def test_empty_operator_breaks_at_once(gpu_ctx):
    """An all-zero operator (nnz = 0): A*v = 0, H(2,1) = 0 at the first step.  BA-GMRES returns
    its zero initial guess (hybrid_ba_gmres_rtp.m:4); AB-RTP leaves x unassigned."""
    A = sp.csr_matrix((6, 4))
    B = sp.csr_matrix(np.ones((4, 6)))
    b, xt = np.arange(1.0, 7.0), np.ones(4)
    g = hgmres.hybrid_ba_gmres_rtp(A, B, b, xt, 0.0, 3, 1e-2, ctx=gpu_ctx)
    r = _oracle(R.hybrid_ba_gmres_rtp, A, B, b, xt, 0.0, 3, 1e-2)
    assert g[3] == r[3]
    for a, b_ in zip(g[:3], r[:3]):
        _same(a, b_)
    with pytest.raises(hgmres.OutputNotAssigned):
        hgmres.hybrid_ab_gmres_rtp(A, B, b, xt, 0.0, 3, 1e-2, ctx=gpu_ctx)


def test_host_spin_default_follows_cpu_affinity(gpu_ctx, tmp_path):
    """ADVICE r4 (host spins): the host waits spin then yield by default, and wait blocking when
    the process may run on fewer than 4 cores (capi.cpp host_spin_default)."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    pkg = os.path.join(ROOT, "hybrid-gmres_amd")
    ncpu = len(os.sched_getaffinity(0))
    assert gpu_ctx.get_option("host_spin_us") == (200 if ncpu >= 4 else -1)
    code = (f"import os, sys; sys.path.insert(0, {pkg!r})\n"
            "os.sched_setaffinity(0, sorted(os.sched_getaffinity(0))[:2])\n"
            "import hgmres\n"
            "print(int(hgmres.Context(0).get_option('host_spin_us')))\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.strip().splitlines()[-1] == "-1"
