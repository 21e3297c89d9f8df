"""ORACLE — CPU restatement of the numeric part of ``analyze_regularization.m`` (test
infrastructure only: imported by ``tests/`` and ``tests/golden/make_golden.py``, never by the
product).

Follows ``analyze_regularization.m:17-49,106-107,122-123`` with the oracle's solvers
(:mod:`oracle.restatement`): the lambda sweep of the hybrid ``*_bounds`` solvers, the GCV
``fminbnd`` per method, the true-optimal lambdas and the final solves.  ``fminbnd`` is
scipy's ``fminbound`` (the same Forsythe-Malcolm-Moler golden-section/parabolic search MATLAB
documents for ``fminbnd``, TolX = xtol) over ``gcv_function`` on one cached Arnoldi (the
reference recomputes the same deterministic Arnoldi at every evaluation).

PARITY STATUS: parity unpinned w.r.t. MATLAB — ``shaw(32)`` is restated from its definition
(``hgmres.regtools``) and MATLAB's ``randn`` stream cannot be reproduced, so the fixture holds
numpy-generated noise and mismatch arrays.
"""
from __future__ import annotations

import numpy as np
import scipy.optimize as so

from . import restatement as R


def analyze_regularization(A, b, x_true, B_pert, DeltaM_AB, DeltaM_BA, *, maxit=32, tol=1e-6,
                           lambda_range=None, k_gcv=20, bounds_outputs=True, explicit_BA=True):
    """``explicit_BA``: BAgmres_nonhybrid_bounds with the formed ``M = B*A`` (``:4``), as the
    reference; False applies ``B*(A*q)`` (the device's order, for the fixed-order parity check)."""
    lam_range = np.logspace(-10, 0, 100) if lambda_range is None else np.asarray(lambda_range)   # :19
    out = {k: np.zeros(lam_range.size) for k in
           ("res_norms_ab", "sol_norms_ab", "err_norms_ab", "res_norms_ba", "sol_norms_ba", "err_norms_ba")}
    nb = np.linalg.norm(b)
    for i, lam in enumerate(lam_range):                                   # :22
        x_ab, err_ab = R.ABgmres_hybrid_bounds(A, B_pert, b, x_true, tol, maxit, lam)[:2]   # :24
        out["res_norms_ab"][i] = np.linalg.norm(b - A @ x_ab) / nb         # :25
        out["sol_norms_ab"][i] = np.linalg.norm(x_ab)                     # :26
        out["err_norms_ab"][i] = err_ab[-1]                               # :27
        x_ba, err_ba = R.BAgmres_hybrid_bounds(A, B_pert, b, x_true, tol, maxit, lam)[:2]   # :29
        out["res_norms_ba"][i] = np.linalg.norm(b - A @ x_ba) / nb         # :30
        out["sol_norms_ba"][i] = np.linalg.norm(x_ba)                     # :31
        out["err_norms_ba"][i] = err_ba[-1]                               # :32
    m = A.shape[0]                                                        # :36
    for side in ("ab", "ba"):
        H, beta = R.arnoldi(A, B_pert, b, k_gcv, side)                    # gcv_function.m:3-33
        trace_m = m if side == "ab" else A.shape[1]
        f = lambda lam: R.gcv_from_H(H, beta, lam, trace_m)
        lam_gcv, g, _, _ = so.fminbound(f, 1e-9, 1e-1, xtol=1e-8, full_output=True)   # :37-40 / :45-46
        out[f"lambda_gcv_{side}"] = float(lam_gcv)
        out[f"gcv_min_{side}"] = float(g)
        idx = int(np.argmin(out[f"err_norms_{side}"]))                     # :41 / :47
        out[f"lambda_true_optimal_{side}"] = lam_range[idx]               # :42 / :48
        out[f"min_err_{side}"] = out[f"err_norms_{side}"][idx]
    dab = DeltaM_AB if bounds_outputs else None
    dba = DeltaM_BA if bounds_outputs else None
    rab = R.ABgmres_hybrid_bounds(A, B_pert, b, x_true, tol, maxit, out["lambda_gcv_ab"], dab)   # :106
    rba = R.BAgmres_hybrid_bounds(A, B_pert, b, x_true, tol, maxit, out["lambda_gcv_ba"], dba)   # :107
    nab = R.ABgmres_nonhybrid_bounds(A, B_pert, b, x_true, tol, maxit, dab)                       # :122
    nba = R.BAgmres_nonhybrid_bounds(A, B_pert, b, x_true, tol, maxit, dba, explicit_BA=explicit_BA)   # :123
    out["x_optimal_ab"], out["x_optimal_ba"] = rab[0], rba[0]
    out["solution_nonhybrid_ab"], out["solution_nonhybrid_ba"] = nab[0], nba[0]
    if bounds_outputs:                  # outputs 5-8 of the final solves (the reference computes them too)
        for key, r in (("opt_ab", rab), ("opt_ba", rba), ("non_ab", nab), ("non_ba", nba)):
            out[f"phi_final_{key}"] = np.real(r[4])
            out[f"dphi_final_{key}"] = np.real(r[5])
            out[f"niters_{key}"] = r[3]
    out["lambda_range"] = lam_range
    return out
