"""The numeric pipeline of ``analyze_regularization.m`` over the device solvers.

``analyze_regularization.m`` is the consumer the north star requires to "see identical
outputs" (SURVEY.md §3.4, §8(f)2).  This module runs its numeric part, with the figures
left out, through the same entry points a MATLAB caller would reach (``*_bounds`` and the GCV
split ``hgm_arnoldi`` + ``hgm_gcv_fminbnd``):

* the 100-point lambda sweep of ``ABgmres_hybrid_bounds`` / ``BAgmres_hybrid_bounds`` with the
  relative residual, solution norm and last error of each solve (``:19-33``);
* the GCV lambda of each method by ``fminbnd`` over ``gcv_function`` on [1e-9, 1e-1], TolX 1e-8
  (``:35-49``).  ``gcv_function`` re-runs the same deterministic Arnoldi at every evaluation, so
  one Arnoldi and the lambda-dependent part on its H give the same values (``plot_gcv_surface.m:58-122``);
* the "true optimal" lambdas (argmin of the error curves, ``:41-42,47-48``);
* the final solves at the GCV lambdas and the non-hybrid solves (``:106-107,122-123``).

The problem set-up of ``:3-15`` (``shaw(32)``, ``randn`` noise, the mismatch ``E``) is
:func:`regularization_problem`; MATLAB's ``rng(0); randn`` cannot be reproduced here, so the
noise comes from numpy and the golden fixture stores the arrays.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import core
from .regtools import generate_test_problem


@dataclass
class RegularizationProblem:
    A: np.ndarray
    b: np.ndarray
    b_exact: np.ndarray
    x_true: np.ndarray
    E: np.ndarray
    B_pert: np.ndarray       # A' + E
    DeltaM_AB: np.ndarray    # A * E
    DeltaM_BA: np.ndarray    # E * A


def regularization_problem(n: int = 32, problem: str = "shaw", noise_level: float = 1e-2,
                           mismatch: float = 1e-4, seed: int = 0) -> RegularizationProblem:
    """``analyze_regularization.m:3-15`` (numpy's generator in place of ``rng(0); randn``)."""
    A, b_exact, x_true = generate_test_problem(problem, n)     # :5
    rng = np.random.default_rng(seed)                          # :7
    noise = rng.standard_normal(b_exact.shape)                 # :9
    noise = noise / np.linalg.norm(noise) * noise_level * np.linalg.norm(b_exact)   # :10
    b = b_exact + noise                                        # :11
    E = mismatch * rng.standard_normal(A.T.shape)              # :12
    B_pert = A.T + E                                           # :13
    return RegularizationProblem(A, b, b_exact, x_true, E, B_pert, A @ E, E @ A)   # :14-15


def analyze_regularization(P: RegularizationProblem, *, maxit: int = 32, tol: float = 1e-6,
                           lambda_range=None, k_gcv: int = 20, ctx=None, DeltaM_factored: bool = False) -> dict:
    """Numeric outputs of ``analyze_regularization.m`` (no figures).

    ``DeltaM_factored``: pass DeltaM as the factor pair (A, E) / (E, A) instead of the
    formed product (the at-scale form; the bounds outputs used here do not depend on it)."""
    ctx = ctx or core.default_context()
    lam_range = np.logspace(-10, 0, 100) if lambda_range is None else np.asarray(lambda_range, dtype=np.float64)
    A = core.as_operator(P.A, ctx)                             # uploaded once, reused by every solve
    Bp = core.as_operator(P.B_pert, ctx)
    dm_ab = (P.A, P.E) if DeltaM_factored else P.DeltaM_AB
    dm_ba = (P.E, P.A) if DeltaM_factored else P.DeltaM_BA
    nb = np.linalg.norm(P.b)
    out = {k: np.zeros(lam_range.size) for k in
           ("res_norms_ab", "sol_norms_ab", "err_norms_ab", "res_norms_ba", "sol_norms_ba", "err_norms_ba")}
    for i, lam in enumerate(lam_range):                        # :22-33
        x_ab, err_ab = core.ABgmres_hybrid_bounds(A, Bp, P.b, P.x_true, tol, maxit, lam, ctx=ctx)[:2]   # :24
        out["res_norms_ab"][i] = np.linalg.norm(P.b - P.A @ x_ab) / nb                                  # :25
        out["sol_norms_ab"][i] = np.linalg.norm(x_ab)                                                   # :26
        out["err_norms_ab"][i] = err_ab[-1]                                                             # :27
        x_ba, err_ba = core.BAgmres_hybrid_bounds(A, Bp, P.b, P.x_true, tol, maxit, lam, ctx=ctx)[:2]   # :29
        out["res_norms_ba"][i] = np.linalg.norm(P.b - P.A @ x_ba) / nb                                  # :30
        out["sol_norms_ba"][i] = np.linalg.norm(x_ba)                                                   # :31
        out["err_norms_ba"][i] = err_ba[-1]                                                             # :32
    m = P.A.shape[0]                                           # :36
    for side in ("ab", "ba"):                                  # :39-40 / :45-46
        H, beta, _ = core.arnoldi(A, Bp, P.b, k_gcv, side, ctx=ctx)
        trace_m = m if side == "ab" else P.A.shape[1]          # gcv_function.m:46-50
        lam_gcv, g = core.gcv_fminbnd(H, beta, trace_m, 1e-9, 1e-1, 1e-8)
        out[f"lambda_gcv_{side}"] = lam_gcv
        out[f"gcv_min_{side}"] = g
        idx = int(np.argmin(out[f"err_norms_{side}"]))          # :41 / :47  [min_err, idx] = min(err_norms)
        out[f"lambda_true_optimal_{side}"] = lam_range[idx]    # :42 / :48
        out[f"min_err_{side}"] = out[f"err_norms_{side}"][idx]
    out["x_optimal_ab"] = core.ABgmres_hybrid_bounds(A, Bp, P.b, P.x_true, tol, maxit, out["lambda_gcv_ab"],
                                                     dm_ab, ctx=ctx)[0]          # :106
    out["x_optimal_ba"] = core.BAgmres_hybrid_bounds(A, Bp, P.b, P.x_true, tol, maxit, out["lambda_gcv_ba"],
                                                     dm_ba, ctx=ctx)[0]          # :107
    out["solution_nonhybrid_ab"] = core.ABgmres_nonhybrid_bounds(A, Bp, P.b, P.x_true, tol, maxit, dm_ab,
                                                                 ctx=ctx)[0]     # :122
    out["solution_nonhybrid_ba"] = core.BAgmres_nonhybrid_bounds(A, Bp, P.b, P.x_true, tol, maxit, dm_ba,
                                                                 ctx=ctx)[0]     # :123
    out["lambda_range"] = lam_range
    return out
