"""The 1-D test problems of ``generate_test_problem.m:1-11`` (Regularization Tools).

The reference calls P. C. Hansen's Regularization Tools (``shaw``, ``deriv2``, ``heat``), which
it does not vendor (version unpinned).  ``shaw`` feeds
``analyze_regularization.m:3-5``, ``plot_gcv_surface.m``, ``plot_filter_factors.m`` and
``plot_perturbation_bound_validation.m``; ``deriv2`` feeds ``run_equivalence_plots.m:4`` and
``run_ptr_rtp_comparison.m:5``.  Both have published closed forms, restated here from their
definitions (Hansen, "Regularization Tools", Numer. Algorithms 6 (1994); the discretisations
below are the ones that package documents):

* ``shaw(n)``: 1-D image restoration, first-kind Fredholm equation on [-pi/2, pi/2] with
  kernel ``K(s,t) = (cos s + cos t)^2 (sin u / u)^2``, ``u = pi (sin s + sin t)``, discretised by
  the midpoint rule on n points (``A(i,j) = h K(s_i, t_j)``, ``h = pi/n``; n even), and the
  two-Gaussian solution ``x(t) = 2 exp(-6 (t - 0.8)^2) + exp(-2 (t + 0.5)^2)``, ``b = A x``.
  The symmetric kernel is evaluated on the upper half only and mirrored, as the package does.
* ``deriv2(n)`` (example 1): second-derivative Green's function ``K(s,t) = s (t-1)`` for
  ``s < t`` and ``t (s-1)`` otherwise on [0,1]^2, Galerkin with box functions (closed-form
  cell integrals), ``x(t) = t``, ``b(s) = (s^3 - s)/6`` projected on the same boxes.

* ``heat(n, kappa=1)``: inverse heat equation, a first-kind Volterra equation on [0,1] with the
  convolution kernel ``k(t) = t^(-3/2) / (2 kappa sqrt(pi)) exp(-1/(4 kappa^2 t))``, collocated at
  the midpoints ``t_i = (i - 1/2) h`` (``h = 1/n``) with the midpoint rule: ``A`` is the lower
  triangular Toeplitz matrix with first column ``h k(t_i)``.  The solution is the package's
  piecewise profile on the first half (``t_i = 20 i / n``: ``0.75 t^2/4`` below 2,
  ``0.75 + (t-2)(3-t)`` below 3, ``0.75 exp(-2 (t-3))`` after) and zero on the second half,
  ``b = A x`` (n even).  Used by ``plot_error_vs_mismatch_norm.m``.

Parity: the arrays are MATLAB's up to rounding in the kernel evaluation order; no MATLAB
output exists to pin them bitwise ("parity unpinned w.r.t. MATLAB's shaw/deriv2/heat").  The tests
check them against their definitions (direct kernel evaluation, quadrature of the cell
integrals, the heat equation's convolution structure).  This is host-side input generation, not part of the timed path.
"""
from __future__ import annotations

import math

import numpy as np


def shaw(n: int):
    """``[A, b, x] = shaw(n)`` (Regularization Tools), dense ``n x n``."""
    if n % 2:
        raise ValueError("The order n must be even")
    h = math.pi / n
    A = np.zeros((n, n))
    s = -math.pi / 2 + (np.arange(n) + 0.5) * h
    co = np.cos(s)
    psi = math.pi * np.sin(s)
    for i in range(n // 2):                       # the upper half, mirrored through the anti-diagonal
        for j in range(i, n - i - 1):
            ss = psi[i] + psi[j]
            A[i, j] = ((co[i] + co[j]) * math.sin(ss) / ss) ** 2
            A[n - j - 1, n - i - 1] = A[i, j]
        A[i, n - i - 1] = (2 * co[i]) ** 2        # psi_i + psi_{n-i+1} = 0: the limit sin(u)/u -> 1
    A = A + np.triu(A, 1).T
    A = A * h
    x = 2.0 * np.exp(-6.0 * (s - 0.8) ** 2) + 1.0 * np.exp(-2.0 * (s + 0.5) ** 2)
    b = A @ x
    return A, b, x


def deriv2(n: int):
    """``[A, b, x] = deriv2(n)`` (example 1), dense ``n x n``."""
    h = 1.0 / n
    sqh = math.sqrt(h)
    h32 = h * sqh
    h2 = h * h
    A = np.zeros((n, n))
    for i in range(1, n + 1):
        A[i - 1, i - 1] = h2 * ((i * i - i + 0.25) * h - (i - 2.0 / 3.0))
        for j in range(1, i):
            A[i - 1, j - 1] = h2 * (j - 0.5) * ((i - 0.5) * h - 1)
    A = A + np.tril(A, -1).T
    i = np.arange(1, n + 1, dtype=np.float64)
    b = h32 * (i - 0.5) * ((i * i + (i - 1) ** 2) * h2 / 2 - 1) / 6
    x = h32 * (i - 0.5)
    return A, b, x


def heat(n: int, kappa: float = 1.0):
    """``[A, b, x] = heat(n, kappa)`` (Regularization Tools; kappa = 1 as generate_test_problem.m:6
    calls it), dense ``n x n`` lower-triangular Toeplitz."""
    if n % 2:
        raise ValueError("The order n must be even")   # x(n/2+1:n) needs an integer n/2
    h = 1.0 / n
    t = (np.arange(n) + 0.5) * h
    c = h / (2.0 * kappa * math.sqrt(math.pi))
    d = 1.0 / (4.0 * kappa * kappa)
    k = c * t ** (-1.5) * np.exp(-d / t)
    idx = np.arange(n)
    A = np.where(idx[:, None] >= idx[None, :], k[np.abs(idx[:, None] - idx[None, :])], 0.0)
    x = np.zeros(n)
    for i in range(1, n // 2 + 1):
        ti = i * 20.0 / n
        if ti < 2:
            x[i - 1] = 0.75 * ti * ti / 4
        elif ti < 3:
            x[i - 1] = 0.75 + (ti - 2) * (3 - ti)
        else:
            x[i - 1] = 0.75 * math.exp(-(ti - 3) * 2)
    b = A @ x
    return A, b, x


def generate_test_problem(name: str, n: int):
    """``[A, b_exact, x_true] = generate_test_problem(name, n)`` (generate_test_problem.m:1-11)."""
    key = name.lower()
    if key == "shaw":
        return shaw(n)
    if key == "deriv2":
        return deriv2(n)
    if key == "heat":
        return heat(n)
    raise ValueError("Unknown problem name. Use shaw, heat, or deriv2.")
