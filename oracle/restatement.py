"""ORACLE — CPU restatement of the reference MATLAB solvers (test infrastructure only).

This module is the checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.

Each function restates one reference ``.m`` file line by line, in numpy/scipy,
with the reference file:line cited beside each step.  MATLAB semantics kept
(SURVEY.md Appendix A):

* operator order ``B*(A*v) + lambda*v`` (two roundings for the epilogue);
* modified Gram–Schmidt with the *updated* ``v`` in each inner product;
* normalisation by division (``v / H(k+1,k)``), breakdown on exact ``== 0``
  (``< 1e-12`` in ``gcv_function.m:30``);
* ``mldivide``: square symmetric with positive diagonal -> Cholesky, falling
  back to LU; rectangular -> Householder QR least squares (:func:`mldivide`);
* histories pre-allocated to ``maxit`` and truncated to ``1:niters``;
  ``niters = k`` even after a breakdown ``break``;
* MATLAB "output argument not assigned" errors raised as ``UnboundLocalError``-
  like :class:`OutputNotAssigned`.

PARITY STATUS: **parity unpinned** with respect to reference artefacts.  The
reference is MATLAB (absent from this image and the GPU box), ships no tests,
fixtures or golden vectors, and depends on un-vendored Regularization Tools /
``PRtomo_mismatched``.  The restatement is instead
cross-checked against independent implementations of the same published
algorithms (``scipy.sparse.linalg.lsqr`` / ``lsmr``, a dense Krylov least-squares
solve) and against the equivalences the reference itself asserts in
``run_equivalence_plots.m:12-22`` and ``run_ptr_rtp_comparison.m:15-19``
(see ``tests/test_oracle.py``).

FIXED-ORDER MODE (:func:`fixed_order`): MATLAB's own summation orders (MKL-blocked
``ddot``/``dnrm2``, its sparse ``mtimes``) cannot be reproduced by any other
implementation, so parity at the ulp level needs one documented order that both sides
follow.  Inside ``with fixed_order():`` every inner product and 2-norm of this module
sums its terms in the order of :func:`_fsum` (64-term chunks left to right, then 64-value
chunks of those, then the rest left to right), ``Q*y`` sums over the columns left to
right, and the Gram products ``AQk'*AQk`` / ``AQk'*b`` are inner products of that kind.
Sparse products stay scipy's (each CSR row, and each ``A.T @ u`` output, summed
sequentially in stored order).  libhgmres' parity mode (``HGM_OPT_PARITY``) runs the same
orders on the GPU, so the two agree to the last bit on the Krylov recurrences.
"""
from __future__ import annotations

import contextlib
import time

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp

EPS = np.finfo(np.float64).eps
_FIXED = False      # fixed-order mode (fixed_order())
_FIX_CH = 64        # chunk length of _fsum (kernels.hip FIX_CH)


class OutputNotAssigned(RuntimeError):
    """MATLAB: 'Output argument "x" not assigned during call'."""


# Iteration clock (bench.py cpu_baseline): while `iteration_clock()` is active, every solver loop
# appends time.perf_counter() at the top of each iteration, so the caller can time the setup
# (before the first tick) apart from the iterations.  No effect on any result.
_CLOCK = None


def _tick():
    if _CLOCK is not None:
        _CLOCK.append(time.perf_counter())


@contextlib.contextmanager
def iteration_clock():
    global _CLOCK
    prev, _CLOCK = _CLOCK, []
    try:
        yield _CLOCK
    finally:
        _CLOCK = prev


@contextlib.contextmanager
def fixed_order(on=True):
    """Run the restatement with the documented fixed summation order (module docstring)."""
    global _FIXED
    prev, _FIXED = _FIXED, bool(on)
    try:
        yield
    finally:
        _FIXED = prev


def _fsum(p):
    """Fixed-order sum of the terms p (each already rounded): level 1 sums 64-term chunks
    left to right, level 2 sums 64-value chunks of those left to right, then the level-2
    values left to right.  np.cumsum is a sequential accumulation; padding with +0.0 does not
    change a sum.  Mirrors kernels.hip k_fixed_l1 / k_fixed_l2."""
    p = np.ascontiguousarray(p, dtype=np.float64).ravel()
    if p.size == 0:
        return 0.0
    for _ in range(2):
        r = (-p.size) % _FIX_CH
        if r:
            p = np.concatenate([p, np.zeros(r)])
        p = np.cumsum(p.reshape(-1, _FIX_CH), axis=1)[:, -1]
    return float(np.cumsum(p)[-1])


def _norm(v):
    # numpy scalars, not Python floats: a division by a zero norm gives MATLAB's Inf / NaN
    # (e.g. beta = 0 for b = 0, norm(x_true) = 0) instead of raising ZeroDivisionError
    if _FIXED:
        v = np.asarray(v, dtype=np.float64)
        return np.float64(np.sqrt(_fsum(v * v)))
    return np.float64(np.linalg.norm(v))


def _dot(a, b):
    """Inner product a'*b (``Q(:,j)'*v``)."""
    if _FIXED:
        return np.float64(_fsum(np.asarray(a, dtype=np.float64) * np.asarray(b, dtype=np.float64)))
    return np.float64(a @ b)


def _gemv(Q, y):
    """``Q*y`` for a dense basis: in fixed-order mode ((Q0 y0 + Q1 y1) + Q2 y2) + ..."""
    if not _FIXED:
        return Q @ y
    x = Q[:, 0] * y[0]
    for j in range(1, Q.shape[1]):
        x = x + Q[:, j] * y[j]
    return x


def _tmat(M, v):
    """``M'*v`` for a dense tall M (one inner product per column)."""
    if not _FIXED:
        return M.T @ v
    return np.array([_dot(M[:, j], v) for j in range(M.shape[1])])


def _gram(M):
    """``M'*M`` for a dense tall M."""
    if not _FIXED:
        return M.T @ M
    k = M.shape[1]
    G = np.empty((k, k))
    for i in range(k):
        for j in range(k):
            G[i, j] = _dot(M[:, i], M[:, j])
    return G


# ---- the k x k kernels in the documented order (fixed-order mode) -------------------------
# MATLAB's `\` is LAPACK (MKL), whose operation order is not specified either.  In
# fixed-order mode the small dense solves follow one documented order: the unblocked
# right-looking forms below (Cholesky R'R = M column by column, LU with partial pivoting,
# Householder QR with column pivoting), each multiply and subtract rounded on its own.
# libhgmres' host code (csrc/dense.cpp) runs the same loops.
def _chol_solve_fixed(M, b):
    n = len(b)
    R = [[float(M[i, j]) for j in range(n)] for i in range(n)]
    for j in range(n):
        s = R[j][j]
        for k in range(j):
            s = s - R[k][j] * R[k][j]
        if not s > 0:
            return None
        rjj = float(np.sqrt(s))
        R[j][j] = rjj
        for i in range(j + 1, n):
            t = R[j][i]
            for k in range(j):
                t = t - R[k][j] * R[k][i]
            R[j][i] = t / rjj
    z = [float(v) for v in b]
    for i in range(n):                       # R' z = b
        t = z[i]
        for k in range(i):
            t = t - R[k][i] * z[k]
        z[i] = t / R[i][i]
    x = [0.0] * n
    for i in range(n - 1, -1, -1):           # R x = z
        t = z[i]
        for k in range(i + 1, n):
            t = t - R[i][k] * x[k]
        x[i] = t / R[i][i]
    return np.array(x)


def _lu_solve_fixed(M, b):
    n = len(b)
    A = [[float(M[i, j]) for j in range(n)] for i in range(n)]
    r = [float(v) for v in b]
    for k in range(n):
        p, best = k, abs(A[k][k])
        for i in range(k + 1, n):
            if abs(A[i][k]) > best:
                best, p = abs(A[i][k]), i
        if p != k:
            A[k], A[p] = A[p], A[k]
            r[k], r[p] = r[p], r[k]
        piv = A[k][k]
        for i in range(k + 1, n):
            lik = A[i][k] / piv
            A[i][k] = lik
            for j in range(k + 1, n):
                A[i][j] = A[i][j] - lik * A[k][j]
            r[i] = r[i] - lik * r[k]
    x = [0.0] * n
    for i in range(n - 1, -1, -1):
        t = r[i]
        for j in range(i + 1, n):
            t = t - A[i][j] * x[j]
        x[i] = t / A[i][i]
    return np.array(x)


def _qr_ls_fixed(M, b):
    m, n = M.shape
    A = [[float(M[i, j]) for i in range(m)] for j in range(n)]   # columns
    r = [float(v) for v in b]
    piv = list(range(n))
    cn = []
    for j in range(n):
        s = 0.0
        for i in range(m):
            s = s + A[j][i] * A[j][i]
        cn.append(s)
    kmax = min(m, n)
    for k in range(kmax):
        p = k
        for j in range(k + 1, n):
            if cn[j] > cn[p]:
                p = j
        if p != k:
            A[k], A[p] = A[p], A[k]
            piv[k], piv[p] = piv[p], piv[k]
            cn[k], cn[p] = cn[p], cn[k]
        alpha = 0.0
        for i in range(k, m):
            alpha = alpha + A[k][i] * A[k][i]
        alpha = float(np.sqrt(alpha))
        if alpha == 0:
            continue
        x0 = A[k][k]
        beta = -alpha if x0 > 0 else alpha
        v0 = x0 - beta
        v = [1.0] + [A[k][i] / v0 for i in range(k + 1, m)]
        tau = (beta - x0) / beta
        A[k][k] = beta
        for i in range(k + 1, m):
            A[k][i] = 0.0
        for j in range(k + 1, n):
            s = 0.0
            for i in range(k, m):
                s = s + v[i - k] * A[j][i]
            s = s * tau
            for i in range(k, m):
                A[j][i] = A[j][i] - s * v[i - k]
        s = 0.0
        for i in range(k, m):
            s = s + v[i - k] * r[i]
        s = s * tau
        for i in range(k, m):
            r[i] = r[i] - s * v[i - k]
        for j in range(k + 1, n):
            s = 0.0
            for i in range(k + 1, m):
                s = s + A[j][i] * A[j][i]
            cn[j] = s
    z = [0.0] * n
    for i in range(kmax - 1, -1, -1):
        t = r[i]
        for j in range(i + 1, kmax):
            t = t - A[j][i] * z[j]
        d = A[i][i]
        z[i] = t / d if d != 0 else 0.0
    y = np.empty(n)
    for j in range(n):
        y[piv[j]] = z[j]
    return y


def _gram_small(Hk):
    """``Hk'*Hk`` of a small dense matrix, each entry summed over the rows in order."""
    r, k = Hk.shape
    G = np.empty((k, k))
    for i in range(k):
        for j in range(k):
            s = 0.0
            for q in range(r):
                s = s + float(Hk[q, i]) * float(Hk[q, j])
            G[i, j] = s
    return G


def _matmul_small(X, Y):
    """``X*Y`` of small dense matrices, each entry summed over the inner index in order."""
    n, p = X.shape[0], Y.shape[1]
    Z = np.empty((n, p))
    for i in range(n):
        for j in range(p):
            s = 0.0
            for q in range(X.shape[1]):
                s = s + float(X[i, q]) * float(Y[q, j])
            Z[i, j] = s
    return Z


def mldivide(M, rhs):
    """MATLAB ``M \\ rhs`` for the small dense systems the solvers form.

    Square + symmetric + positive diagonal -> Cholesky (falls back to LU when
    not positive definite); square otherwise -> LU; rectangular -> QR least
    squares with column pivoting (LAPACK xGEQP3, as MATLAB).  In fixed-order mode
    the same three factorisations run in their documented loop order."""
    M = np.asarray(M, dtype=np.float64)
    rhs = np.asarray(rhs, dtype=np.float64)
    r, c = M.shape
    if _FIXED:
        if r != c:
            return _qr_ls_fixed(M, rhs)
        if np.array_equal(M, M.T) and np.all(np.diag(M) > 0):
            x = _chol_solve_fixed(M, rhs)
            if x is not None:
                return x
        return _lu_solve_fixed(M, rhs)
    if r == c:
        if np.array_equal(M, M.T) and np.all(np.diag(M) > 0):
            try:
                cf = sla.cho_factor(M, lower=False, check_finite=False)
                return sla.cho_solve(cf, rhs, check_finite=False)
            except np.linalg.LinAlgError:
                pass
        return sla.solve(M, rhs, check_finite=False)
    Qm, R, piv = sla.qr(M, mode="economic", pivoting=True, check_finite=False)
    z = sla.solve_triangular(R, Qm.T @ rhs, check_finite=False)
    y = np.empty_like(z)
    y[piv] = z
    return y


def _mgs_arnoldi_step(Q, H, k, v, breakdown_tol=None):
    """Arnoldi MGS inner loop, ``hybrid_ba_gmres_rtp.m:20-26`` (0-based k).
    Returns True on breakdown."""
    for j in range(k + 1):                       # :20  for j = 1:k
        H[j, k] = _dot(Q[:, j], v)               # :21  H(j,k) = Q(:,j)'*v
        v = v - H[j, k] * Q[:, j]                # :22  v = v - H(j,k)*Q(:,j)
    H[k + 1, k] = _norm(v)                       # :24  H(k+1,k) = norm(v)
    if breakdown_tol is None:
        if H[k + 1, k] == 0:                     # :25  if H(k+1,k) == 0, break
            return True
    elif H[k + 1, k] < breakdown_tol:            # gcv_function.m:30
        return True
    Q[:, k + 1] = v / H[k + 1, k]                # :26  Q(:,k+1) = v / H(k+1,k)
    return False


def _cgs2_arnoldi_step(Q, H, k, v, breakdown_tol=None):
    """Classical Gram-Schmidt applied twice in place of MGS (BASELINE configs[2]'s option; the
    reference itself only has MGS, hybrid_ba_gmres_rtp.m:20-23): h1 = Q'v, v -= Q h1,
    h2 = Q'v, v -= Q h2, H(1:k,k) = h1 + h2; normalisation and breakdown as :24-26."""
    Qk = Q[:, : k + 1]
    h1 = _tmat(Qk, v)
    v = v - _gemv(Qk, h1)
    h2 = _tmat(Qk, v)
    v = v - _gemv(Qk, h2)
    H[: k + 1, k] = h1 + h2
    H[k + 1, k] = _norm(v)
    if breakdown_tol is None:
        if H[k + 1, k] == 0:
            return True
    elif H[k + 1, k] < breakdown_tol:
        return True
    Q[:, k + 1] = v / H[k + 1, k]
    return False


def _arnoldi_step(Q, H, k, v, breakdown_tol=None, orth="mgs"):
    if orth == "cgs2":
        return _cgs2_arnoldi_step(Q, H, k, v, breakdown_tol)
    return _mgs_arnoldi_step(Q, H, k, v, breakdown_tol)


def hybrid_ba_gmres_rtp(A, B, b, x_true, tol, maxit, lam, return_H=False, orth="mgs"):
    """``hybrid_ba_gmres_rtp.m:1-42``."""
    n = A.shape[1]                               # :3
    x = np.zeros(n)                              # :4
    M_reg = lambda v: B @ (A @ v) + lam * v      # :6
    d = B @ b                                    # :7
    r0 = d - M_reg(x)                            # :9
    beta = _norm(r0)                             # :10
    Q = np.zeros((n, maxit + 1))                 # :11
    H = np.zeros((maxit + 1, maxit))             # :12
    Q[:, 0] = r0 / beta                          # :13
    error_norm = np.zeros(maxit)                 # :15
    residual_norm = np.zeros(maxit)              # :16
    nb, nxt = _norm(b), _norm(x_true)
    k = 0
    for k in range(maxit):                       # :18
        _tick()
        v = M_reg(Q[:, k])                       # :19
        if _arnoldi_step(Q, H, k, v, orth=orth): # :20-26
            break
        Hk = H[: k + 2, : k + 1]                 # :28
        rhs = np.zeros(k + 2)
        rhs[0] = beta
        yk = mldivide(Hk, rhs)                   # :29
        x = _gemv(Q[:, : k + 1], yk)             # :30
        residual_norm[k] = _norm(b - A @ x) / nb     # :32
        error_norm[k] = _norm(x - x_true) / nxt      # :33
        if residual_norm[k] <= tol:              # :35
            break
    niters = k + 1                               # :38
    out = (x, error_norm[:niters], residual_norm[:niters], niters)
    return out + (H,) if return_H else out


def hybrid_ab_gmres_rtp(A, B, b, x_true, tol, maxit, lam, return_H=False):
    """``hybrid_ab_gmres_rtp.m:1-45`` (n-space Arnoldi on B*A + lambda*I)."""
    n = A.shape[1]                               # :3
    x0 = np.zeros(n)                             # :4
    M_reg_op = lambda v: B @ (A @ v) + lam * v   # :6
    d_krylov = B @ b                             # :7
    r0 = d_krylov - M_reg_op(x0)                 # :9
    beta = _norm(r0)                             # :10
    Q = np.zeros((n, maxit + 1))                 # :11
    H = np.zeros((maxit + 1, maxit))             # :12
    Q[:, 0] = r0 / beta                          # :13
    error_norm = np.zeros(maxit)
    residual_norm = np.zeros(maxit)
    nb, nxt = _norm(b), _norm(x_true)
    x = None
    k = 0
    for k in range(maxit):                       # :18
        _tick()
        v = M_reg_op(Q[:, k])                    # :19
        if _mgs_arnoldi_step(Q, H, k, v):        # :20-26
            break
        Qk = Q[:, : k + 1]                       # :28
        AQk = A @ Qk                             # :31
        G = _gram(AQk)
        yk = mldivide(G + lam * np.eye(k + 1), _tmat(AQk, b))   # :32
        x = _gemv(Qk, yk)                        # :33
        residual_norm[k] = _norm(b - A @ x) / nb     # :35
        error_norm[k] = _norm(x - x_true) / nxt      # :36
        if residual_norm[k] <= tol:              # :38
            break
    if x is None:                                # breakdown at k=1: x never assigned
        raise OutputNotAssigned('Output argument "x" not assigned (hybrid_ab_gmres_rtp)')
    niters = k + 1                               # :41
    out = (x, error_norm[:niters], residual_norm[:niters], niters)
    return out + (H,) if return_H else out


def lsqr_solver(A, b, x_true, tol, maxit):
    """``lsqr_solver.m:1-54``."""
    n = A.shape[1]
    x = np.zeros(n)                              # :5
    beta = _norm(b)                              # :7
    u = b / beta                                 # :8
    v_hat = A.T @ u                              # :10
    alpha = _norm(v_hat)                         # :11
    v = v_hat / alpha                            # :12
    w = v.copy()                                 # :14
    phi_bar = beta                               # :15
    rho_bar = alpha                              # :16
    error_norm = np.zeros(maxit)
    residual_norm = np.zeros(maxit)
    nb, nxt = _norm(b), _norm(x_true)
    k = 0
    for k in range(maxit):                       # :20
        _tick()
        u_hat = A @ v - alpha * u                # :22
        beta = _norm(u_hat)                      # :23
        u = u_hat / beta                         # :24
        v_hat = A.T @ u - beta * v               # :26
        alpha = _norm(v_hat)                     # :27
        v = v_hat / alpha                        # :28
        rho = np.sqrt(rho_bar ** 2 + beta ** 2)  # :31
        c = rho_bar / rho                        # :32
        s = beta / rho                           # :33
        theta = s * alpha                        # :35
        rho_bar = -c * alpha                     # :36
        phi = c * phi_bar                        # :37
        phi_bar = s * phi_bar                    # :38
        x = x + (phi / rho) * w                  # :40
        w = v - (theta / rho) * w                # :41
        error_norm[k] = _norm(x - x_true) / nxt  # :43
        residual_norm[k] = abs(phi_bar) / nb     # :44
        if residual_norm[k] <= tol:              # :46
            break
    niters = k + 1                               # :49
    error_norm = error_norm[:niters]
    residual_norm = residual_norm[:niters].copy()
    residual_norm[-1] = _norm(b - A @ x) / nb    # :52
    return x, error_norm, residual_norm, niters


def lsmr_solver(A, b, x_true=None, tol=None, maxit=None):
    """``lsmr_solver.m:1-83`` (defaults ``:3,5``)."""
    if tol is None:
        tol = 1e-6                               # :3
    m, n = A.shape                               # :4
    if maxit is None:
        maxit = min(m, n)                        # :5
    x = np.zeros(n)                              # :7
    u = b.copy()                                 # :10
    beta = _norm(u)                              # :11
    if beta > 0:
        u = u / beta                             # :12
    v = A.T @ u                                  # :14
    alpha = _norm(v)                             # :15
    if alpha > 0:
        v = v / alpha                            # :16
    zetabar = alpha * beta                       # :19
    alphabar = alpha                             # :20
    rho = 1.0                                    # :21
    rhobar = 1.0                                 # :22
    cbar, sbar = 1.0, 0.0                        # :23
    h = v.copy()                                 # :25
    hbar = np.zeros(n)                           # :26
    err_hist = np.full(maxit, np.nan)            # :28
    res_hist = np.zeros(maxit)                   # :29
    ar_hist = np.zeros(maxit)                    # :30
    nb = _norm(b)
    if hasattr(A, "fro_norm"):                   # operator wrappers used by the tests
        normA = A.fro_norm()
    elif _FIXED and sp.issparse(A):              # norm(A,'fro') over the stored values
        normA = _norm(sp.csr_matrix(A).data)
    else:
        normA = float(sp.linalg.norm(A, "fro")) if sp.issparse(A) else float(np.linalg.norm(A, "fro"))
    k = 0
    for k in range(maxit):                       # :32
        _tick()
        u = A @ v - alpha * u                    # :34
        beta = _norm(u)                          # :35
        if beta > 0:
            u = u / beta                         # :36
        v = A.T @ u - beta * v                   # :38
        alpha = _norm(v)                         # :39
        if alpha > 0:
            v = v / alpha                        # :40
        alphahat = alphabar                      # :42
        rhoold = rho                             # :43
        rho = np.hypot(alphahat, beta)           # :44
        c = alphahat / rho                       # :45
        s = beta / rho                           # :46
        thetanew = s * alpha                     # :48
        alphabar = c * alpha                     # :49
        rhobarold = rhobar                       # :51
        thetabar = sbar * rho                    # :52
        rhobar = np.hypot(cbar * rho, thetanew)  # :53
        cbar = (cbar * rho) / rhobar             # :54
        sbar = thetanew / rhobar                 # :55
        zeta = cbar * zetabar                    # :58
        zetabar = -sbar * zetabar                # :59
        if k == 0:
            hbar = h.copy()                      # :62
        else:
            hbar = h - (thetabar * rho) / (rhoold * rhobarold) * hbar   # :64
        x = x + (zeta / (rho * rhobar)) * hbar   # :66
        h = v - (thetanew / rho) * h             # :67
        r = b - A @ x                            # :69
        res_hist[k] = _norm(r) / (nb + EPS)      # :70
        ar_hist[k] = _norm(A.T @ r) / (normA * max(_norm(r), EPS))   # :71
        if x_true is not None and np.size(x_true) > 0:
            err_hist[k] = _norm(x - x_true) / _norm(x_true)           # :72-73
        if res_hist[k] < tol:                    # :76
            break
    iters = k + 1                                # :79
    return x, err_hist[:iters], res_hist[:iters], ar_hist[:iters], iters


def hybrid_lsqr_solver(A, b, x_true, tol, maxit, lam):
    """``hybrid_lsqr_solver.m:1-52`` (explicit augmentation ``:5-6``)."""
    m, n = A.shape
    if hasattr(A, "augment"):                    # operator wrappers used by the tests
        A_aug = A.augment(lam)
    else:
        A_aug = sp.vstack([sp.csr_matrix(A), np.sqrt(lam) * sp.identity(n, format="csr")]).tocsr()   # :5
    b_aug = np.concatenate([b, np.zeros(n)])     # :6
    x = np.zeros(n)                              # :8
    beta_aug = _norm(b_aug)                      # :9
    u_aug = b_aug / beta_aug                     # :10
    v_hat = A_aug.T @ u_aug                      # :11
    alpha_aug = _norm(v_hat)                     # :12
    v = v_hat / alpha_aug                        # :13
    w = v.copy()                                 # :14
    phi_bar = beta_aug                           # :15
    rho_bar = alpha_aug                          # :16
    error_norm = np.zeros(maxit)
    residual_norm = np.zeros(maxit)
    nb, nxt = _norm(b), _norm(x_true)
    k = 0
    for k in range(maxit):                       # :21
        u_hat = A_aug @ v - alpha_aug * u_aug    # :22
        beta_aug = _norm(u_hat)                  # :23
        u_aug = u_hat / beta_aug                 # :24
        v_hat = A_aug.T @ u_aug - beta_aug * v   # :26
        alpha_aug = _norm(v_hat)                 # :27
        v = v_hat / alpha_aug                    # :28
        rho = np.sqrt(rho_bar ** 2 + beta_aug ** 2)   # :30
        c = rho_bar / rho                        # :31
        s = beta_aug / rho                       # :32
        theta = s * alpha_aug                    # :34
        rho_bar = -c * alpha_aug                 # :35
        phi = c * phi_bar                        # :36
        phi_bar = s * phi_bar                    # :37
        x = x + (phi / rho) * w                  # :39
        w = v - (theta / rho) * w                # :40
        error_norm[k] = _norm(x - x_true) / nxt  # :42
        residual_norm[k] = _norm(b - A @ x) / nb # :43
        if residual_norm[k] < tol:               # :45
            break
    niters = k + 1
    return x, error_norm[:niters], residual_norm[:niters], niters


def hybrid_lsmr_solver(A, b, x_true, tol, maxit, lam):
    """``hybrid_lsmr_solver.m:1-57``."""
    n = A.shape[1]
    x = np.zeros(n)                              # :4
    u = b.copy()                                 # :6
    beta1 = _norm(u)                             # :7
    u = u / beta1                                # :8
    V = np.zeros((n, maxit))                     # :10
    B_k = np.zeros((maxit + 1, maxit))           # :11
    v_hat = A.T @ u                              # :13
    alpha1 = _norm(v_hat)                        # :14
    v = v_hat / alpha1                           # :15
    V[:, 0] = v                                  # :16
    error_norm = np.zeros(maxit)
    residual_norm = np.zeros(maxit)
    nb, nxt = _norm(b), _norm(x_true)
    k = 0
    for k in range(maxit):                       # :21
        B_k[k, k] = alpha1                       # :23
        u_hat = A @ v - alpha1 * u               # :24
        beta_k = _norm(u_hat)                    # :25
        u = u_hat / beta_k                       # :26
        B_k[k + 1, k] = beta_k                   # :27
        if k < maxit - 1:                        # :29
            v_hat = A.T @ u - beta_k * v         # :30
            alpha_k_plus_1 = _norm(v_hat)        # :31
            v = v_hat / alpha_k_plus_1           # :32
            V[:, k + 1] = v                      # :33
            alpha1 = alpha_k_plus_1              # :34
        Bk = B_k[: k + 2, : k + 1]               # :37
        alpha_k1 = alpha1                        # :38
        beta_k1 = beta_k                         # :39
        G = _gram_small(Bk) if _FIXED else Bk.T @ Bk
        E11 = np.zeros((k + 1, k + 1))
        E11[0, 0] = 1.0
        GG = _matmul_small(G, G) if _FIXED else G @ G
        LHS = GG + (alpha_k1 * beta_k1) ** 2 * E11 + lam * np.eye(k + 1)   # :41
        e1 = np.zeros(k + 1)
        e1[0] = 1.0
        RHS = B_k[0, 0] * beta1 * (G[:, 0].copy() if _FIXED else G @ e1)   # :42
        yk = mldivide(LHS, RHS)                  # :44
        x = _gemv(V[:, : k + 1], yk)             # :45
        error_norm[k] = _norm(x - x_true) / nxt  # :47
        residual_norm[k] = _norm(b - A @ x) / nb # :48
        if residual_norm[k] <= tol:              # :50
            break
    niters = k + 1
    return x, error_norm[:niters], residual_norm[:niters], niters


def _dense(M):
    return M.toarray() if sp.issparse(M) else np.asarray(M, dtype=np.float64)


def _spectrum(A, B, side):
    """``M = A*B`` / ``B*A``; ``[U,D] = eig(M)``; real parts sorted descending with the
    eigenvector columns (*_bounds.m:4-9).  Dense: small problems only."""
    M = _dense(A) @ _dense(B) if side == "ab" else _dense(B) @ _dense(A)   # :4
    D, U = np.linalg.eig(M)                      # :6-7 (LAPACK dgeev: unit 2-norm vectors)
    mu_full = np.real(D)                         # :8 / :7
    order = np.argsort(-mu_full, kind="stable")  # sort(mu_full, 'descend')
    return mu_full[order], U[:, order]


def _filter_iteration(H, Q, k, mu_full, UA, DeltaM, lam, side, hybrid):
    """phi / dphi of iteration k (1-based): ABgmres_hybrid_bounds.m:43-78,
    ABgmres_nonhybrid_bounds.m:42-73, BAgmres_hybrid_bounds.m:42-74,
    BAgmres_nonhybrid_bounds.m:42-74."""
    Qk = Q[:, :k]                                # :43 / :42
    DM = _dense(DeltaM)
    dK = Qk.T @ (DM @ Qk)                        # :44 / :43  Qk'*DeltaM*Qk
    Hs = H[:k, :k]                               # :46 / :43-45
    ek = np.zeros(k)
    ek[-1] = 1.0                                 # :47
    if side == "ba" and hybrid:
        Hf = H[: k + 1, :k]                      # BA hybrid :44
        Th, W = sla.eig(Hf.T @ Hf, Hs)           # :46  eig(Hk_full'*Hk_full, Hk_small)
    else:
        X = np.zeros((k, k))
        X[:, -1] = mldivide(Hs.T, ek)            # Hk_small' \ (ek*ek'): only the last column
        P = Hs + (H[k, k - 1] ** 2) * X          # AB :48 / nonhybrid :48 / :47
        if hybrid:
            P = P + lam * np.eye(k)              # AB hybrid :49
        Th, W = np.linalg.eig(P)                 # :50 / :49 / :48
    Theta = np.real(Th)                          # :51 / :50 / :49
    p_sort = np.argsort(Theta, kind="stable")    # :52  sort(Theta)
    Theta = Theta[p_sort]
    W = W[:, p_sort]                             # :53
    dTheta = np.real(np.einsum("ij,ik,kj->j", W.conj(), dK, W))   # :55  real(diag(W'*dK*W))
    dMu = np.sum(UA[:, :k] * (DM @ UA[:, :k]), axis=0).conj()     # :56  sum(UA.*(DeltaM*UA),1)'
    mu = mu_full[:k]                             # :58
    s2l = mu + lam if hybrid else mu             # :60 (hybrid); nonhybrid uses mu
    eps0 = EPS                                   # :61
    Clog = np.zeros(k)
    P_excl = np.zeros((k, k))
    for i in range(k):                           # :64-71
        terms = np.maximum(1 - s2l[i] / Theta, eps0)
        Clog[i] = np.sum(np.log(terms))
        for j in range(k):
            denom = max(1 - s2l[i] / Theta[j], eps0)
            P_excl[i, j] = np.exp(Clog[i] - np.log(denom))
    P_final = np.exp(Clog)                       # :72
    if hybrid:
        phi = (mu / s2l) * (1 - P_final)         # :73
        term1 = -mu * np.sum((dTheta / Theta ** 2) * P_excl, axis=1)            # :75
        term2 = (lam / s2l ** 2) * (1 - P_final) * dMu                           # :76
        term3 = (mu / s2l) * np.sum((1 / Theta) * P_excl, axis=1) * dMu          # :77
        dphi = term1 + term2 + term3             # :78
    else:
        phi = 1 - P_final                        # nonhybrid :69
        term1 = -mu * np.sum((dTheta / Theta ** 2) * P_excl, axis=1)            # :71
        term2 = np.sum((1 / Theta) * P_excl, axis=1) * dMu                      # :72
        dphi = term1 + term2                     # :73
    return phi, dphi


def _gmres_ptr(A, B, b, x_true, tol, maxit, lam, side, hybrid, explicit_BA=False, return_H=False,
               DeltaM=None, return_Q=False):
    """Arnoldi + projected-solve part of ``{AB,BA}gmres_{hybrid,nonhybrid}_bounds.m``
    (lines cited per variant below).  With ``DeltaM`` the spectral-bound outputs 5-8
    (``phi_final, dphi_final, phi_iter, dphi_iter``) follow the reference's dense
    ``eig(M)`` (small problems only); the GPU computes them from Ritz pairs at scale."""
    m, n = A.shape
    spec = _spectrum(A, B, side) if DeltaM is not None else None
    phi_iter, dphi_iter = [], []
    if side == "ab":
        r0 = b - A @ (B @ np.zeros(B.shape[1]))  # AB*_bounds.m:11-12
        dim = m
        op = lambda q: A @ (B @ q)               # AB*_bounds.m:25
    else:
        if hybrid:
            r0 = B @ (b - A @ np.zeros(n))       # BAgmres_hybrid_bounds.m:12-13
            op = lambda q: B @ (A @ q)           # BAgmres_hybrid_bounds.m:25
        else:
            r0 = B @ b                           # BAgmres_nonhybrid_bounds.m:12-13
            if explicit_BA:
                M = (B @ A)                      # BAgmres_nonhybrid_bounds.m:4
                op = lambda q: M @ q             # :25
            else:
                op = lambda q: B @ (A @ q)
        dim = n
    beta = _norm(r0)
    Q = np.zeros((dim, maxit + 1))
    H = np.zeros((maxit + 1, maxit))
    Q[:, 0] = r0 / beta
    res = np.zeros(maxit)
    err = np.zeros(maxit)
    nb, nxt = _norm(b), _norm(x_true)
    xk = None
    k = 0
    for k in range(maxit):                       # :24
        _tick()
        v = op(Q[:, k])                          # :25
        if _mgs_arnoldi_step(Q, H, k, v):        # :26-32
            break
        Hk = H[: k + 2, : k + 1]
        tk = np.zeros(k + 2)
        tk[0] = beta
        if hybrid:
            if _FIXED:                           # tk = beta e1: Hk'*tk = beta Hk(1,:)'
                yk = mldivide(_gram_small(Hk) + lam * np.eye(k + 1), Hk[0, :] * beta)   # hybrid :34-36
            else:
                yk = mldivide(Hk.T @ Hk + lam * np.eye(k + 1), Hk.T @ tk)   # hybrid :34-36
        else:
            yk = mldivide(Hk, tk)                # nonhybrid :35
        zk = _gemv(Q[:, : k + 1], yk)            # :37 / :36
        xk = B @ zk if side == "ab" else zk      # AB :38 ; BA :37
        res[k] = _norm(b - A @ xk) / nb          # :40 / :39
        err[k] = _norm(xk - x_true) / nxt        # :41 / :40
        if spec is not None:                     # :42-81
            ph, dph = _filter_iteration(H, Q, k + 1, spec[0], spec[1], DeltaM, lam, side, hybrid)
            phi_iter.append(ph)
            dphi_iter.append(dph)
        if res[k] <= tol:                        # :83 / :78 / :79
            break
    if xk is None:
        raise OutputNotAssigned('Output argument "x" not assigned (*gmres_*_bounds)')
    niters = k + 1
    out = (xk, err[:niters], res[:niters], niters)
    if spec is not None:
        # phi_final = phi_iter{k}: empty when iteration k broke down before :80
        last = phi_iter[-1] if len(phi_iter) == niters else np.zeros(0)
        dlast = dphi_iter[-1] if len(dphi_iter) == niters else np.zeros(0)
        out = out + (last, dlast, phi_iter, dphi_iter)
    if return_H:
        out = out + (H,)
    if return_Q:
        out = out + (Q,)
    return out


def ABgmres_hybrid_bounds(A, B, b, x_true, tol, maxit, lam, DeltaM=None, return_H=False, return_Q=False):
    """``ABgmres_hybrid_bounds.m:1-96`` (outputs 5-8 when ``DeltaM`` is given)."""
    return _gmres_ptr(A, B, b, x_true, tol, maxit, lam, "ab", True, return_H=return_H, DeltaM=DeltaM,
                      return_Q=return_Q)


def ABgmres_nonhybrid_bounds(A, B, b, x_true, tol, maxit, DeltaM=None, return_H=False, return_Q=False):
    """``ABgmres_nonhybrid_bounds.m:1-91``."""
    return _gmres_ptr(A, B, b, x_true, tol, maxit, 0.0, "ab", False, return_H=return_H, DeltaM=DeltaM,
                      return_Q=return_Q)


def BAgmres_hybrid_bounds(A, B, b, x_true, tol, maxit, lam, DeltaM=None, return_H=False, return_Q=False):
    """``BAgmres_hybrid_bounds.m:1-92``."""
    return _gmres_ptr(A, B, b, x_true, tol, maxit, lam, "ba", True, return_H=return_H, DeltaM=DeltaM,
                      return_Q=return_Q)


def BAgmres_nonhybrid_bounds(A, B, b, x_true, tol, maxit, DeltaM=None, explicit_BA=True, return_H=False,
                             return_Q=False):
    """``BAgmres_nonhybrid_bounds.m:1-92`` — uses the explicit product
    ``M = B*A`` as the reference does (``:4,25``)."""
    return _gmres_ptr(A, B, b, x_true, tol, maxit, 0.0, "ba", False,
                      explicit_BA=explicit_BA, return_H=return_H, DeltaM=DeltaM, return_Q=return_Q)


def arnoldi(A, B, b, k_gcv, gcv_type, breakdown_tol=1e-12, orth="mgs"):
    """Arnoldi part of ``gcv_function.m:3-33``: returns (H, beta) with H of
    size (k_gcv+1) x k_gcv (zero columns kept after a break, ``:33``)."""
    if gcv_type == "ab":
        r0 = b                                   # :5
        dim = A.shape[0]
        op = lambda q: A @ (B @ q)               # :20
    else:
        r0 = B @ b                               # :8
        dim = A.shape[1]
        op = lambda q: B @ (A @ q)               # :22
    beta = _norm(r0)                             # :12
    Q = np.zeros((dim, k_gcv + 1))               # :13
    H = np.zeros((k_gcv + 1, k_gcv))             # :14
    Q[:, 0] = r0 / beta                          # :15
    for k in range(k_gcv):                       # :18
        _tick()
        v = op(Q[:, k])
        if _arnoldi_step(Q, H, k, v, breakdown_tol=breakdown_tol, orth=orth):   # :25-31
            break
    return H, beta


def gcv_from_H(H, beta, lam, trace_m):
    """λ-dependent part of ``gcv_function.m:33-58`` on a cached H."""
    k = H.shape[1]                               # :33
    Hk = H[: k + 1, :k]                          # :35
    tk = np.zeros(k + 1)
    tk[0] = beta                                 # :16,:36
    yk = mldivide(Hk.T @ Hk + lam * np.eye(k), Hk.T @ tk)   # :38
    residual_norm_sq = _norm(tk - Hk @ yk) ** 2  # :40
    s_diag = np.linalg.svd(H[:k, :k], compute_uv=False)     # :42-43
    trace_val = np.sum(s_diag ** 2 / (s_diag ** 2 + lam))   # :51
    denominator = (trace_m - trace_val) ** 2     # :52
    with np.errstate(divide="ignore", invalid="ignore"):
        gcv_val = residual_norm_sq / denominator  # :54
    if np.isnan(gcv_val) or np.isinf(gcv_val) or denominator < EPS:   # :56
        gcv_val = 1e20                           # :57
    return float(gcv_val)


def gcv_function(lam, A, B, b, m, k_gcv, gcv_type):
    """``gcv_function.m:1-59``."""
    H, beta = arnoldi(A, B, b, k_gcv, gcv_type)
    trace_m = m if gcv_type == "ab" else A.shape[1]   # :46-50
    return gcv_from_H(H, beta, lam, trace_m)


# ---------------------------------------------------------------------------------------------
# fp32 Golub-Kahan (BASELINE configs[4]: lsqr_solver / lsmr_solver with a single-precision
# operator and single-precision Krylov vectors).  The reference is fp64 MATLAB; this is its
# algorithm line by line (cited) in the arithmetic libhgmres' fp32 path uses, in the documented
# fixed order:
#   * operator and vectors in float32 (b, x_true rounded to float32 once);
#   * products summed sequentially per row in float32 (scipy csr_matvec<float>, or
#     oracle/parallel.py's float32 OpenMP product: the same bits);
#   * sums of squares / differences in float32 in the fixed order of _fsum32;
#   * the scalars (beta, alpha, the rotations) in double from those float32 sums, and every
#     scalar that scales a vector rounded to float32 first;
#   * ||A||_F (lsmr_solver.m:71) in double over the float32 values, fixed order.
# libhgmres in parity mode (HGM_OPT_PARITY) on an HGM_F32 operator runs exactly this, so the
# two agree bit for bit (tests/test_gpu_parity_mode.py).
# ---------------------------------------------------------------------------------------------
f32 = np.float32


_F32_SUM = (64, False)   # (chunk, reversed) of _fsum32: (64, False) is the documented fixed order


@contextlib.contextmanager
def fsum32_order(chunk, reverse):
    """_fsum32 in ANOTHER fixed order (chunk length, terms reversed) -- test infrastructure: the
    fp32 oracle's own rounding spread over correct fp32 orders (tests/golden/make_golden.py
    dump_c5).  Never used by the parity checks."""
    global _F32_SUM
    prev, _F32_SUM = _F32_SUM, (int(chunk), bool(reverse))
    try:
        yield
    finally:
        _F32_SUM = prev


def _fsum32(p):
    """_fsum's order (64-term chunks, then 64-value chunks of those, then left to right) with
    every partial sum rounded to float32 (np.cumsum accumulates in the array's dtype)."""
    p = np.ascontiguousarray(p, dtype=np.float32).ravel()
    if p.size == 0:
        return f32(0.0)
    ch, rev = _F32_SUM
    if rev:
        p = p[::-1]
    for _ in range(2):
        r = (-p.size) % ch
        if r:
            p = np.concatenate([p, np.zeros(r, dtype=np.float32)])
        p = np.cumsum(p.reshape(-1, ch), axis=1, dtype=np.float32)[:, -1]
    return f32(np.cumsum(p, dtype=np.float32)[-1])


def _nrm32(v):
    """norm(v) of a float32 vector: sqrt in double of the float32 fixed-order sum of squares."""
    v = np.asarray(v, dtype=np.float32)
    return np.float64(np.sqrt(np.float64(_fsum32(v * v))))


def _nrm32_diff(a, b):
    d = np.asarray(a, dtype=np.float32) - np.asarray(b, dtype=np.float32)
    return np.float64(np.sqrt(np.float64(_fsum32(d * d))))


def _op32(A):
    """(A*v, A'*u) of a float32 operator: scipy CSR float32 (or a ParallelCSR of one)."""
    if hasattr(A, "dtype") and not sp.issparse(A):
        return A, A.T
    A = sp.csr_matrix(A, dtype=np.float32)
    return A, A.T


def _mv32(M, v):
    y = M @ np.asarray(v, dtype=np.float32)
    assert y.dtype == np.float32
    return y


def lsqr_solver_f32(A, b, x_true, tol, maxit):
    """``lsqr_solver.m:1-54`` with a float32 operator and float32 vectors (see the section note)."""
    A, At = _op32(A)
    n = A.shape[1]
    b32, xt32 = np.asarray(b, dtype=np.float32), np.asarray(x_true, dtype=np.float32)
    x = np.zeros(n, dtype=np.float32)            # :5
    nb = _nrm32(b32)
    nxt = _nrm32_diff(xt32, x)
    beta = nb                                    # :7
    u = b32 / f32(beta)                          # :8
    v_hat = _mv32(At, u)                         # :10
    alpha = _nrm32(v_hat)                        # :11
    v = v_hat / f32(alpha)                       # :12
    w = v.copy()                                 # :14
    phi_bar, rho_bar = beta, alpha               # :15-16
    error_norm = np.zeros(maxit)
    residual_norm = np.zeros(maxit)
    k = 0
    for k in range(maxit):                       # :20
        _tick()
        u_hat = _mv32(A, v) - f32(alpha) * u     # :22
        beta = _nrm32(u_hat)                     # :23
        u = u_hat / f32(beta)                    # :24
        v_hat = _mv32(At, u) - f32(beta) * v     # :26
        alpha = _nrm32(v_hat)                    # :27
        v = v_hat / f32(alpha)                   # :28
        rho = np.sqrt(rho_bar * rho_bar + beta * beta)   # :31
        c = rho_bar / rho                        # :32
        s = beta / rho                           # :33
        theta = s * alpha                        # :35
        rho_bar = -c * alpha                     # :36
        phi = c * phi_bar                        # :37
        phi_bar = s * phi_bar                    # :38
        x = x + f32(phi / rho) * w               # :40
        w = v - f32(theta / rho) * w             # :41
        error_norm[k] = _nrm32_diff(x, xt32) / nxt   # :43
        residual_norm[k] = abs(phi_bar) / nb     # :44
        if residual_norm[k] <= tol:              # :46
            break
    niters = k + 1                               # :49
    error_norm = error_norm[:niters]
    residual_norm = residual_norm[:niters].copy()
    r = b32 - _mv32(A, x)
    residual_norm[-1] = _nrm32(r) / nb           # :52
    return x, error_norm, residual_norm, niters


def lsmr_solver_f32(A, b, x_true=None, tol=None, maxit=None):
    """``lsmr_solver.m:1-83`` with a float32 operator and float32 vectors (section note)."""
    A, At = _op32(A)
    if tol is None:
        tol = 1e-6                               # :3
    m, n = A.shape                               # :4
    if maxit is None:
        maxit = min(m, n)                        # :5
    b32 = np.asarray(b, dtype=np.float32)
    have_xt = x_true is not None and np.size(x_true) > 0
    xt32 = np.asarray(x_true, dtype=np.float32) if have_xt else None
    x = np.zeros(n, dtype=np.float32)            # :7
    nb = _nrm32(b32)
    nxt = _nrm32_diff(xt32, x) if have_xt else 0.0
    vals = A.val if hasattr(A, "val") else sp.csr_matrix(A).data
    normA = np.sqrt(_fsum(np.asarray(vals, dtype=np.float32).astype(np.float64) ** 2))   # :71 norm(A,'fro')
    u = b32.copy()                               # :10
    beta = nb                                    # :11
    if beta > 0:
        u = u / f32(beta)                        # :12
    v = _mv32(At, u)                             # :14
    alpha = _nrm32(v)                            # :15
    if alpha > 0:
        v = v / f32(alpha)                       # :16
    zetabar = alpha * beta                       # :19
    alphabar = alpha                             # :20
    rho, rhobar, cbar, sbar = 1.0, 1.0, 1.0, 0.0 # :21-23
    h = v.copy()                                 # :25
    hbar = np.zeros(n, dtype=np.float32)         # :26
    err_hist = np.full(maxit, np.nan)            # :28
    res_hist = np.zeros(maxit)                   # :29
    ar_hist = np.zeros(maxit)                    # :30
    k = 0
    for k in range(maxit):                       # :32
        _tick()
        u = _mv32(A, v) - f32(alpha) * u         # :34
        beta = _nrm32(u)                         # :35
        if beta > 0:
            u = u / f32(beta)                    # :36
        v = _mv32(At, u) - f32(beta) * v         # :38
        alpha = _nrm32(v)                        # :39
        if alpha > 0:
            v = v / f32(alpha)                   # :40
        alphahat = alphabar                      # :42
        rhoold = rho                             # :43
        rho = np.hypot(alphahat, beta)           # :44
        c = alphahat / rho                       # :45
        s = beta / rho                           # :46
        thetanew = s * alpha                     # :48
        alphabar = c * alpha                     # :49
        rhobarold = rhobar                       # :51
        thetabar = sbar * rho                    # :52
        rhobar = np.hypot(cbar * rho, thetanew)  # :53
        cbar = (cbar * rho) / rhobar             # :54
        sbar = thetanew / rhobar                 # :55
        zeta = cbar * zetabar                    # :58
        zetabar = -sbar * zetabar                # :59
        if k == 0:
            hbar = h.copy()                      # :62
        else:
            hbar = h - f32((thetabar * rho) / (rhoold * rhobarold)) * hbar   # :64
        x = x + f32(zeta / (rho * rhobar)) * hbar   # :66
        h = v - f32(thetanew / rho) * h          # :67
        r = b32 - _mv32(A, x)                    # :69
        nr = _nrm32(r)
        res_hist[k] = nr / (nb + EPS)            # :70
        ar_hist[k] = _nrm32(_mv32(At, r)) / (normA * max(nr, EPS))   # :71
        if have_xt:
            err_hist[k] = _nrm32_diff(x, xt32) / nxt                   # :72-73
        if res_hist[k] < tol:                    # :76
            break
    iters = k + 1                                # :79
    return x, err_hist[:iters], res_hist[:iters], ar_hist[:iters], iters
