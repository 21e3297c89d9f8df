"""Oracle (CPU restatement of the reference .m files) checked before it is trusted.

The reference ships no fixtures and cannot run here (MATLAB absent), so the
restatement is pinned by (a) independent implementations of the same published
algorithms (scipy's LSQR / LSMR / damped LSQR, a dense Krylov least-squares
solve), (b) the equivalences the reference itself asserts in
run_equivalence_plots.m:12-22 and run_ptr_rtp_comparison.m:15-19, and (c) the
committed golden fixtures (tests/golden/make_golden.py).
"""
import numpy as np
import pytest
import scipy.optimize as so
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from conftest import golden_problem, load_golden
from hgmres.problems import tomo_problem
from oracle import restatement as R


def rel(a, b):
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-300)


@pytest.fixture(scope="module")
def P64():
    return tomo_problem(64, 90, noise=1e-2, seed=0)


@pytest.fixture(scope="module")
def P24():
    return tomo_problem(24, 12, noise=1e-2, seed=0)


# ---- (a) independent implementations -------------------------------------------------
def test_lsqr_matches_scipy(P64):
    A, b, xt = P64.A, P64.b, P64.x_true
    for k in (1, 5, 10):
        x = R.lsqr_solver(A, b, xt, 0.0, k)[0]
        xs = spla.lsqr(A, b, atol=0, btol=0, conlim=0, iter_lim=k)[0]
        assert rel(x, xs) < 1e-8, k


def test_lsmr_matches_scipy(P64):
    A, b, xt = P64.A, P64.b, P64.x_true
    for k in (1, 5, 10):
        x = R.lsmr_solver(A, b, xt, 0.0, k)[0]
        xs = spla.lsmr(A, b, atol=0, btol=0, conlim=0, maxiter=k)[0]
        assert rel(x, xs) < 1e-8, k


def test_hybrid_lsqr_matches_damped_lsqr(P64):
    A, b, xt = P64.A, P64.b, P64.x_true
    lam = 1e-2
    x = R.hybrid_lsqr_solver(A, b, xt, 0.0, 8, lam)[0]
    xs = spla.lsqr(A, b, damp=np.sqrt(lam), atol=0, btol=0, conlim=0, iter_lim=8)[0]
    assert rel(x, xs) < 1e-8


def test_ba_gmres_is_krylov_least_squares(P24):
    """x_k = argmin ||B b - (BA) x|| over K_k(BA, Bb), by a dense independent solve."""
    A, B, b, xt = P24.A, P24.B, P24.b, P24.x_true
    k = 6
    x = R.BAgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k)[0]
    M = (B @ A).toarray()
    d = B @ b
    K = np.zeros((M.shape[0], k))
    q = d / np.linalg.norm(d)
    for j in range(k):
        K[:, j] = q
        q = M @ q
        q /= np.linalg.norm(q)
    Qk, _ = np.linalg.qr(K)
    y = np.linalg.lstsq(M @ Qk, d, rcond=None)[0]
    assert rel(x, Qk @ y) < 1e-8


def test_mldivide_branches():
    rng = np.random.default_rng(0)
    G = rng.standard_normal((6, 6))
    S = G @ G.T + 6 * np.eye(6)
    r = rng.standard_normal(6)
    assert rel(R.mldivide(S, r), np.linalg.solve(S, r)) < 1e-12          # Cholesky
    N = G + 0.0
    assert rel(R.mldivide(N, r), np.linalg.solve(N, r)) < 1e-12          # LU
    H = rng.standard_normal((7, 6))
    r7 = rng.standard_normal(7)
    assert rel(R.mldivide(H, r7), np.linalg.lstsq(H, r7, rcond=None)[0]) < 1e-12   # QR LS


# ---- (b) the reference's own equivalence claims (B = A') -------------------------------
def test_equivalences_run_equivalence_plots(P64):
    A, B, b, xt = P64.A, P64.B, P64.b, P64.x_true
    k, lam = 8, 1e-3
    x_ba = R.BAgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k)[0]
    x_lsmr = R.lsmr_solver(A, b, xt, 0.0, k)[0]
    assert rel(x_ba, x_lsmr) < 1e-7            # run_equivalence_plots.m:12-13, title :33 (≡)
    x_ab = R.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k)[0]
    x_lsqr = R.lsqr_solver(A, b, xt, 0.0, k)[0]
    assert rel(x_ab, x_lsqr) < 1e-7            # :15-16, title :44 (≡)
    x_hab = R.ABgmres_hybrid_bounds(A, B, b, xt, 0.0, k, lam)[0]
    x_hlsqr = R.hybrid_lsqr_solver(A, b, xt, 0.0, k, lam)[0]
    assert rel(x_hab, x_hlsqr) > 1e-6          # :21-22, title :66 (≠)


def test_hybrid_ba_vs_hybrid_lsmr_is_not_equivalent_as_written(P64):
    """run_equivalence_plots.m:55 titles hybrid BA-GMRES ≡ hybrid LSMR, but the k x k
    system of hybrid_lsmr_solver.m:41-44 is not the PTR normal equations; the
    restatement exposes the gap (documented in DESIGN.md)."""
    A, B, b, xt = P64.A, P64.B, P64.b, P64.x_true
    x1 = R.BAgmres_hybrid_bounds(A, B, b, xt, 0.0, 8, 1e-3)[0]
    x2 = R.hybrid_lsmr_solver(A, b, xt, 0.0, 8, 1e-3)[0]
    assert rel(x1, x2) > 1e-6


def test_ptr_ne_rtp(P64):
    """run_ptr_rtp_comparison.m:15-19, sgtitle :42."""
    A, B, b, xt = P64.A, P64.B, P64.b, P64.x_true
    lam = 1e-3
    e_ptr = R.BAgmres_hybrid_bounds(A, B, b, xt, 0.0, 10, lam)[1]
    e_rtp = R.hybrid_ba_gmres_rtp(A, B, b, xt, 0.0, 10, lam)[1]
    assert np.max(np.abs(e_ptr - e_rtp)) > 1e-8
    e_ptr = R.ABgmres_hybrid_bounds(A, B, b, xt, 0.0, 10, lam)[1]
    e_rtp = R.hybrid_ab_gmres_rtp(A, B, b, xt, 0.0, 10, lam)[1]
    assert np.max(np.abs(e_ptr - e_rtp)) > 1e-8


def test_ab_rtp_is_n_space_on_BA_plus_lambda(P24):
    """SURVEY §0 naming quirk: hybrid_ab_gmres_rtp's Arnoldi equals hybrid_ba_gmres_rtp's."""
    A, B, b, xt = P24.A, P24.B, P24.b, P24.x_true
    H1 = R.hybrid_ab_gmres_rtp(A, B, b, xt, 0.0, 8, 1e-2, return_H=True)[4]
    H2 = R.hybrid_ba_gmres_rtp(A, B, b, xt, 0.0, 8, 1e-2, return_H=True)[4]
    assert np.array_equal(H1, H2)


# ---- MATLAB semantics -----------------------------------------------------------------
def test_arnoldi_relation_and_truncation(P24):
    A, B, b, xt = P24.A, P24.B, P24.b, P24.x_true
    x, e, r, k, H = R.hybrid_ba_gmres_rtp(A, B, b, xt, 0.0, 10, 1e-2, return_H=True)
    assert k == 10 and e.shape == (10,) and r.shape == (10,)
    assert np.all(np.triu(H[:, :], -1) == H)          # upper Hessenberg


def test_tol_stop_semantics(P24):
    A, B, b, xt = P24.A, P24.B, P24.b, P24.x_true
    _, _, r_all, _ = R.hybrid_ba_gmres_rtp(A, B, b, xt, 0.0, 12, 1e-2)
    tol = r_all[4]                                   # `<=` stops exactly at k = 5
    _, e, r, k = R.hybrid_ba_gmres_rtp(A, B, b, xt, tol, 12, 1e-2)
    assert k == 5 and r.shape == (5,)
    # lsmr uses `<` (lsmr_solver.m:76)
    _, _, rl, _, _ = R.lsmr_solver(A, b, xt, 0.0, 12)
    _, _, rl2, _, k2 = R.lsmr_solver(A, b, xt, rl[4], 12)
    assert k2 == 6


def test_breakdown_semantics():
    """H(k+1,k)==0 -> break with niters = k; zero history entry kept; AB-RTP has no x."""
    A = sp.csr_matrix(np.diag([1.0, 2.0, 3.0, 4.0]))
    B = A.T.tocsr()
    b = np.array([1.0, 0.0, 0.0, 0.0])     # invariant subspace of B*A of dimension 1
    xt = np.ones(4)
    x, e, r, k = R.hybrid_ba_gmres_rtp(A, B, b, xt, 0.0, 3, 0.0)
    assert k == 1 and r[0] == 0.0 and np.all(x == 0)
    with pytest.raises(R.OutputNotAssigned):
        R.hybrid_ab_gmres_rtp(A, B, b, xt, 0.0, 3, 0.0)
    # exact-arithmetic Krylov dimension 2: B*A = diag(1,1,4,4), B*b = [2,2,2,2]
    A2 = sp.csr_matrix(np.diag([1.0, 1.0, 2.0, 2.0]))
    b2 = np.array([2.0, 2.0, 1.0, 1.0])
    x, e, r, k = R.hybrid_ab_gmres_rtp(A2, A2.T.tocsr(), b2, xt, 0.0, 4, 0.0)
    assert k == 2 and r[1] == 0.0 and e[1] == 0.0 and r[0] > 0


def test_lsmr_defaults_and_nan_err(P24):
    A, b = P24.A, P24.b
    x, eh, rh, ah, it = R.lsmr_solver(A, b)
    assert it <= min(A.shape)
    assert np.all(np.isnan(eh))                       # lsmr_solver.m:28,72 (no x_true)


# ---- GCV -----------------------------------------------------------------------------
def test_gcv_from_cached_H_equals_gcv_function(P24):
    A, B, b = P24.A, P24.B, P24.b
    m = A.shape[0]
    for typ, tm in (("ab", m), ("ba", A.shape[1])):
        H, beta = R.arnoldi(A, B, b, 10, typ)
        for lam in (1e-6, 1e-3, 1e-1):
            assert R.gcv_from_H(H, beta, lam, tm) == R.gcv_function(lam, A, B, b, m, 10, typ)


def test_gcv_fminbnd_oracle_finds_minimum(P24):
    A, B, b = P24.A, P24.B, P24.b
    H, beta = R.arnoldi(A, B, b, 10, "ba")
    f = lambda l: R.gcv_from_H(H, beta, l, A.shape[1])   # noqa: E731
    lo = so.fminbound(f, 1e-9, 1e-1, xtol=1e-8)
    grid = np.logspace(-9, -1, 200)
    assert f(lo) <= min(f(g) for g in grid) * (1 + 1e-6)


# ---- (c) golden fixtures ---------------------------------------------------------------
@pytest.mark.parametrize("name", ["tomo24_matched.npz", "tomo24_pixel.npz"])
def test_oracle_reproduces_golden(name):
    A, B, b, xt, g = golden_problem(name)
    maxit, lam = int(g["maxit"]), float(g["lam"])
    x, e, r, k, H = R.hybrid_ab_gmres_rtp(A, B, b, xt, 0.0, maxit, lam, return_H=True)
    assert k == int(g["hab_k"]) and np.array_equal(H, g["hab_H"]) and np.array_equal(x, g["hab_x"])
    x, e, r, k = R.lsqr_solver(A, b, xt, 0.0, maxit)
    assert np.array_equal(x, g["lsqr_x"]) and np.array_equal(r, g["lsqr_res"])
    x, eh, rh, ah, k = R.lsmr_solver(A, b, xt, 0.0, maxit)
    assert np.array_equal(ah, g["lsmr_ar"])


def test_golden_c1_operator_hash():
    """The generator still produces the operator the C1 fixture was made from."""
    import hashlib
    g = load_golden("tomo64_c1.npz")
    P = tomo_problem(int(g["N"]), int(g["n_angles"]), noise=1e-2, seed=0)
    h = hashlib.sha256()
    for a in (P.A.indptr.astype(np.int64), P.A.indices.astype(np.int32), P.A.data.astype(np.float64)):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == str(g["A_sha256"])
    assert np.array_equal(P.b, g["b"])


# ---- fixed-order mode (the order libhgmres' parity mode follows) --------
def _fsum_loops(p, ch=64):
    """Plain-Python restatement of the fixed order (for checking R._fsum's numpy form)."""
    def level(v):
        out = []
        for i in range(0, len(v), ch):
            s = v[i]
            for t in v[i + 1:i + ch]:
                s = s + t
            out.append(s)
        return out
    c = level([float(t) for t in p])
    d = level(c)
    s = d[0]
    for t in d[1:]:
        s = s + t
    return s


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 4095, 4096, 4097, 70001])
def test_fsum_matches_loop_form(n):
    p = np.random.default_rng(n).standard_normal(n) * np.exp(np.random.default_rng(n + 1).uniform(-20, 20, n))
    assert R._fsum(p) == _fsum_loops(p)
    import math
    assert abs(R._fsum(p) - math.fsum(p)) <= 1e-12 * np.sum(np.abs(p))


def test_fixed_order_switches_only_the_summation_order(P64):
    """Fixed-order solves agree with the default-order restatement to rounding (they are the
    same algorithm), and the mode is scoped to the with-block."""
    A, B, b, xt = P64.A, P64.B.tocsr(), P64.b, P64.x_true
    o1 = R.hybrid_ab_gmres_rtp(A, B, b, xt, 0.0, 12, 1e-2, return_H=True)
    with R.fixed_order():
        assert R._FIXED
        o2 = R.hybrid_ab_gmres_rtp(A, B, b, xt, 0.0, 12, 1e-2, return_H=True)
        l2 = R.lsqr_solver(A, b, xt, 0.0, 6)
    assert not R._FIXED
    assert np.max(np.abs(o1[-1] - o2[-1])) <= 1e-12 * np.max(np.abs(o1[-1]))
    assert rel(o1[0], o2[0]) < 1e-11
    assert rel(R.lsqr_solver(A, b, xt, 0.0, 6)[0], l2[0]) < 1e-9


def test_parallel_oracle_spmv_is_bitwise_scipy(P64):
    """bench.py cpu_baseline's all-core leg: oracle/spmv_omp.c gives scipy's bits."""
    from oracle import parallel as OP
    OP.build()
    A = P64.A.tocsr()
    PA = OP.ParallelCSR(A)
    rng = np.random.default_rng(0)
    v, u = rng.standard_normal(A.shape[1]), rng.standard_normal(A.shape[0])
    assert np.array_equal(PA @ v, A @ v)
    assert np.array_equal(PA.T @ u, A.T @ u)
    assert np.array_equal(R.lsqr_solver(PA, P64.b, P64.x_true, 0.0, 5)[0],
                          R.lsqr_solver(A, P64.b, P64.x_true, 0.0, 5)[0])


def test_fixed_order_dense_kernels_match_lapack():
    """The documented-order k x k solves of fixed_order() (mirrors of csrc/dense.cpp) solve
    the same systems as LAPACK to rounding."""
    rng = np.random.default_rng(4)
    for n in (1, 5, 20):
        X = rng.standard_normal((n + 1, n))
        M = X.T @ X + 1e-2 * np.eye(n)
        b = rng.standard_normal(n)
        assert rel(R._chol_solve_fixed(M, b), np.linalg.solve(M, b)) < 1e-10
        Mn = rng.standard_normal((n, n))
        assert rel(R._lu_solve_fixed(Mn, b), np.linalg.solve(Mn, b)) < 1e-9
        c = rng.standard_normal(n + 1)
        assert rel(R._qr_ls_fixed(X, c), np.linalg.lstsq(X, c, rcond=None)[0]) < 1e-10
    assert R._chol_solve_fixed(np.array([[1.0, 2.0], [2.0, 1.0]]), np.ones(2)) is None   # not PD
