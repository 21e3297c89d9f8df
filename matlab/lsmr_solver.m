function [x, err_hist, res_hist, ar_hist, iters] = lsmr_solver(A, b, x_true, tol, maxit)
% Signature and defaults of the reference's lsmr_solver.m:1-5 (hgm_lsmr_solver on the MI355X).
% An empty x_true leaves err_hist NaN, as lsmr_solver.m:28.
if nargin < 3, x_true = []; end
if nargin < 4 || isempty(tol), tol = 1e-6; end
if nargin < 5 || isempty(maxit), maxit = min(size(A, 1), size(A, 2)); end
[x, err_hist, res_hist, ar_hist, iters] = hgmres_mex('lsmr_solver', A, b, x_true, tol, maxit);
end
