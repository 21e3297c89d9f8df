import sys, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/hybrid-gmres_amd")
import hgmres
from oracle import restatement as R
ctx = hgmres.Context(0)
N, na = 64, 45
R_ = hgmres.SparseOperator.siddon(N, na, ctx=ctx, order="reference")
rng = np.random.default_rng(3)
x = rng.standard_normal(N * N); u = rng.standard_normal(R_.shape[0]); xt = rng.random(N * N)
b = R_ @ xt
A = R_.to_scipy()
xr = R.lsqr_solver(A, b, xt, 0.0, 10)[0]
for order in ["reference", (4, 0), (4, 16), (8, 32)]:
    T = hgmres.SparseOperator.siddon(N, na, ctx=ctx, order=order)
    l = hgmres.lsqr_solver(T, b, xt, 0.0, 10, ctx=ctx)[0]
    print(order, np.linalg.norm(l - xr) / np.linalg.norm(xr))
# perturbation sensitivity of the oracle
bp = b * (1 + 1e-16 * rng.standard_normal(b.size))
xp = R.lsqr_solver(A, bp, xt, 0.0, 10)[0]
print("oracle 1e-16 perturbation:", np.linalg.norm(xp - xr) / np.linalg.norm(xr))
