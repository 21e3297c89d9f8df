"""Filter-factor bounds (outputs 5-8 of *_bounds.m) at scale: time the device path on a
tomography operator with the unmatched pixel-driven back-projector, DeltaM factored as
(A, E) / (E, A) with E = B - A' (never formed), against the plain solve (outputs 1-4).
usage: python scripts/bounds_scale.py N angles maxit ritz_steps"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
import hgmres  # noqa: E402
from hgmres.problems import tomo_problem  # noqa: E402


def main():
    N, na, maxit, p = (int(a) for a in sys.argv[1:5])
    t0 = time.perf_counter()
    P = tomo_problem(N, na, noise=1e-2, seed=0, backprojector="pixel")
    E = (P.B - P.A.T).tocsr()
    ctx = hgmres.Context(0)
    A = hgmres.SparseOperator.from_scipy(P.A, ctx)
    B = hgmres.SparseOperator.from_scipy(P.B, ctx)
    Eo = hgmres.SparseOperator.from_scipy(E, ctx)
    setup = time.perf_counter() - t0
    out = {"N": N, "angles": na, "m": P.A.shape[0], "n": P.A.shape[1], "nnz_A": int(P.A.nnz), "nnz_E": int(E.nnz),
           "maxit": maxit, "ritz_steps": p, "host_setup_s": round(setup, 2)}
    for side, fn, dm in (("ab", hgmres.ABgmres_hybrid_bounds, (A, Eo)), ("ba", hgmres.BAgmres_hybrid_bounds, (Eo, A))):
        fn(A, B, P.b, P.x_true, 0.0, maxit, 1e-2, ctx=ctx)                    # warm-up
        ctx.synchronize()
        t = time.perf_counter()
        base = fn(A, B, P.b, P.x_true, 0.0, maxit, 1e-2, ctx=ctx)
        ctx.synchronize()
        t_solve = time.perf_counter() - t
        t = time.perf_counter()
        full = fn(A, B, P.b, P.x_true, 0.0, maxit, 1e-2, dm, ctx=ctx, ritz_steps=p, return_ritz=True)
        ctx.synchronize()
        t_full = time.perf_counter() - t
        assert np.array_equal(full[0], base[0])
        mu, rr = full[8], full[9]
        out[side] = {"solve_ms": round(t_solve * 1e3, 2), "solve_plus_bounds_ms": round(t_full * 1e3, 2),
                     "niters": full[3], "mu_top5": [float(v) for v in mu[:5]],
                     "ritz_resid_rel_top5": [float(r / mu[0]) for r in rr[:5]],
                     "phi_final_head": [float(v) for v in full[4][:5]],
                     "dphi_final_head": [float(v) for v in full[5][:5]]}
        print(side, out[side], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
