"""CPU checks of the host-side spectral code of the filter-factor bounds (outputs 5-8 of the
four *_bounds.m files; hybrid-gmres_amd/csrc/spectral.cpp) against the oracle's restatement of
the reference's dense eig sequence, and of the restated Regularization-Tools problems.
No GPU: these entry points are pure host code of libhgmres."""
import warnings

import numpy as np
import pytest
from scipy import integrate

import hgmres
from hgmres.problems import tomo_problem
from hgmres.regtools import deriv2, generate_test_problem, heat, shaw
from oracle import restatement as R


def test_eig_matches_lapack():
    rng = np.random.default_rng(1)
    worst = 0.0
    for n in (1, 2, 3, 5, 8, 17, 32, 60):
        for kind in ("general", "symmetric", "hessenberg"):
            M = rng.standard_normal((n, n))
            if kind == "symmetric":
                M = M + M.T
            elif kind == "hessenberg":
                M = np.triu(M, -1)
            w, V = hgmres.eig(M)
            wn = np.linalg.eigvals(M)
            nrm = np.linalg.norm(M, 2)
            worst = max(worst, np.max(np.abs(np.sort_complex(w) - np.sort_complex(wn))) / nrm)
            worst = max(worst, np.max(np.linalg.norm(M @ V - V * w, axis=0)) / nrm)    # M v = lambda v
            worst = max(worst, np.max(np.abs(np.linalg.norm(V, axis=0) - 1)))           # unit 2-norm (dgeev)
    assert worst < 1e-13, worst


@pytest.fixture(scope="module")
def tomo_bounds():
    """24^2 tomography with the unmatched pixel-driven B, DeltaM = A*E with E = B - A'
    (the mismatch the reference studies): k <= 10 keeps the Arnoldi well conditioned."""
    P = tomo_problem(24, 12, noise=1e-2, seed=0, backprojector="pixel")
    E = (P.B - P.A.T).toarray()
    A = P.A.toarray()
    return P, A @ E, E @ A


@pytest.mark.parametrize("side,hybrid", [("ab", 1), ("ab", 0), ("ba", 1), ("ba", 0)])
def test_filter_factors_match_oracle(tomo_bounds, side, hybrid):
    P, dm_ab, dm_ba = tomo_bounds
    dm = dm_ab if side == "ab" else dm_ba
    lam = 1e-2 if hybrid else 0.0
    fn = {("ab", 1): R.ABgmres_hybrid_bounds, ("ab", 0): R.ABgmres_nonhybrid_bounds,
          ("ba", 1): R.BAgmres_hybrid_bounds, ("ba", 0): R.BAgmres_nonhybrid_bounds}[(side, hybrid)]
    args = (P.A, P.B, P.b, P.x_true, 0.0, 10) + ((lam,) if hybrid else ())
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        out = fn(*args, dm, return_H=True, return_Q=True)
    k, phi_iter, dphi_iter, H, Q = out[3], out[6], out[7], out[8], out[9]
    mu_full, UA = R._spectrum(P.A, P.B, side)
    dK = Q[:, :k].T @ (dm @ Q[:, :k])
    worst = 0.0
    for kk in range(1, k + 1):
        dmu = np.real(np.sum(UA[:, :kk] * (dm @ UA[:, :kk]), axis=0))
        phi, dphi = hgmres.filter_factors(H[: kk + 1, :kk], kk, dK[:kk, :kk], mu_full[:kk], dmu, lam, side, hybrid)
        pr, dr = np.real(phi_iter[kk - 1]), np.real(dphi_iter[kk - 1])
        worst = max(worst, np.max(np.abs(phi - pr)) / np.max(np.abs(pr)),
                    np.max(np.abs(dphi - dr)) / np.max(np.abs(dr)))
    print(f"{side} hybrid={hybrid}: max rel |d phi|, |d dphi| = {worst:.2e}")
    assert worst < 1e-9, worst


@pytest.mark.parametrize("side", ["ab", "ba"])
def test_ritz_full_dimension_is_eig(tomo_bounds, side):
    """A full-dimension Arnoldi (with reorthogonalisation) on M: its Ritz pairs are eig(M)."""
    P, dm_ab, dm_ba = tomo_bounds
    A, B = P.A.toarray(), P.B.toarray()
    M = A @ B if side == "ab" else B @ A
    dm = dm_ab if side == "ab" else dm_ba
    dim = M.shape[0]
    rng = np.random.default_rng(3)
    Q = np.zeros((dim, dim + 1))
    Hp = np.zeros((dim + 1, dim))
    q = rng.standard_normal(dim)
    Q[:, 0] = q / np.linalg.norm(q)
    hmax = 0.0
    for j in range(dim):
        v = M @ Q[:, j]
        for _ in range(2):
            h = Q[:, : j + 1].T @ v
            v = v - Q[:, : j + 1] @ h
            Hp[: j + 1, j] += h
        Hp[j + 1, j] = np.linalg.norm(v)
        hmax = max(hmax, np.max(np.abs(Hp[: j + 2, j])))
        if j + 1 < dim:
            if not Hp[j + 1, j] > 1e-12 * hmax:     # invariant subspace (M is rank deficient): deflate
                Hp[j + 1, j] = 0.0
                v = rng.standard_normal(dim)
                for _ in range(2):
                    v = v - Q[:, : j + 1] @ (Q[:, : j + 1].T @ v)
            Q[:, j + 1] = v / np.linalg.norm(v)
    G = Q[:, :dim].T @ dm @ Q[:, :dim]
    nev = 10
    mu, dmu, rr = hgmres.ritz(Hp[:dim, :dim], Hp[dim, dim - 1], G, nev)
    mu_full, UA = R._spectrum(P.A, P.B, side)
    dmu_ref = np.real(np.sum(UA[:, :nev] * (dm @ UA[:, :nev]), axis=0))
    assert np.max(np.abs(mu - mu_full[:nev])) <= 1e-12 * abs(mu_full[0])
    assert np.max(np.abs(dmu - dmu_ref)) <= 1e-9 * np.max(np.abs(dmu_ref)), np.max(np.abs(dmu - dmu_ref))


def test_shaw_matches_its_definition():
    """shaw(n): midpoint collocation of (cos s + cos t)^2 (sin u / u)^2, u = pi (sin s + sin t)."""
    for n in (8, 32, 64):
        A, b, x = shaw(n)
        h = np.pi / n
        s = -np.pi / 2 + (np.arange(n) + 0.5) * h
        S, T = np.meshgrid(s, s, indexing="ij")
        u = np.pi * (np.sin(S) + np.sin(T))
        with np.errstate(all="ignore"):
            sinc = np.where(u == 0, 1.0, np.sin(u) / u)
        K = h * (np.cos(S) + np.cos(T)) ** 2 * sinc ** 2
        assert np.max(np.abs(A - K)) <= 1e-14 * np.max(np.abs(A))
        assert np.array_equal(A, A.T)
        assert np.allclose(x, 2 * np.exp(-6 * (s - 0.8) ** 2) + np.exp(-2 * (s + 0.5) ** 2), rtol=0, atol=1e-15)
        assert np.array_equal(b, A @ x)
    with pytest.raises(ValueError):
        shaw(7)


def test_deriv2_matches_cell_integrals():
    """deriv2(n): Galerkin cell integrals of the Green's function of -u'' on [0,1]."""
    n = 8
    A, b, x = deriv2(n)
    h = 1.0 / n
    K = lambda s, t: s * (t - 1) if s < t else t * (s - 1)
    for i, j in ((3, 1), (7, 2), (2, 6)):
        val, _ = integrate.dblquad(lambda t, s: K(s, t), i * h, (i + 1) * h, j * h, (j + 1) * h, epsabs=1e-14)
        assert abs(A[i, j] - val / h) <= 1e-12 * abs(val / h)
    for i in (0, 5, 7):                        # diagonal cells: the inner integral split at t = s
        lo, hi = i * h, (i + 1) * h
        inner = lambda s: (s - 1) * (s * s - lo * lo) / 2 + s * ((hi - 1) ** 2 - (s - 1) ** 2) / 2
        val, _ = integrate.quad(inner, lo, hi, epsabs=1e-15)
        assert abs(A[i, i] - val / h) <= 1e-12 * abs(val / h)
    for i in (0, 4, 7):
        bv, _ = integrate.quad(lambda s: (s ** 3 - s) / 6, i * h, (i + 1) * h)
        xv, _ = integrate.quad(lambda s: s, i * h, (i + 1) * h)
        assert abs(b[i] - bv / np.sqrt(h)) <= 1e-13 and abs(x[i] - xv / np.sqrt(h)) <= 1e-13
    assert np.array_equal(A, A.T)
    with pytest.raises(ValueError):
        generate_test_problem("nope", 8)


def test_heat_matches_its_definition():
    """heat(n): midpoint collocation of the Volterra kernel k(s - t) = (s-t)^(-3/2)/(2 sqrt(pi))
    exp(-1/(4 (s-t))) (kappa = 1), lower-triangular Toeplitz; the piecewise solution profile."""
    for n in (8, 32, 64):
        A, b, x = heat(n)
        h = 1.0 / n
        t = (np.arange(n) + 0.5) * h
        for i, j in ((0, 0), (n - 1, 0), (n // 2, 3), (n - 1, n - 2)):
            tau = t[i - j]                                # Toeplitz: k at the lag's midpoint
            assert abs(A[i, j] - h * tau ** -1.5 / (2 * np.sqrt(np.pi)) * np.exp(-1 / (4 * tau))) <= 1e-15 * A[i, j] + 1e-300
        assert np.all(np.triu(A, 1) == 0)
        assert all(np.array_equal(np.diag(A, -d), np.full(n - d, A[d, 0])) for d in range(n))
        ti = np.arange(1, n // 2 + 1) * 20.0 / n
        xr = np.where(ti < 2, 0.75 * ti ** 2 / 4, np.where(ti < 3, 0.75 + (ti - 2) * (3 - ti), 0.75 * np.exp(-(ti - 3) * 2)))
        assert np.allclose(x[: n // 2], xr, rtol=1e-15, atol=0) and np.all(x[n // 2:] == 0)
        assert np.array_equal(b, A @ x)
    # generate_test_problem.m:6 dispatches to heat(n)
    A, b, x = generate_test_problem("heat", 32)
    assert np.array_equal(A, heat(32)[0])
    with pytest.raises(ValueError):
        heat(7)
