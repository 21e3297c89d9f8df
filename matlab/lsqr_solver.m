function [x, error_norm, residual_norm, niters] = lsqr_solver(A, b, x_true, tol, maxit)
% Signature of the reference's lsqr_solver.m:1 (hgm_lsqr_solver on the MI355X; A' is formed by
% the device transpose).
[x, error_norm, residual_norm, niters] = hgmres_mex('lsqr_solver', A, b, x_true, tol, maxit);
end
