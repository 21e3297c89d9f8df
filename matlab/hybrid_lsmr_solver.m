function [x, error_norm, residual_norm, niters] = hybrid_lsmr_solver(A, b, x_true, tol, maxit, lambda)
% Signature of the reference's hybrid_lsmr_solver.m:1 (hgm_hybrid_lsmr_solver on the MI355X).
[x, error_norm, residual_norm, niters] = hgmres_mex('hybrid_lsmr_solver', A, b, x_true, tol, maxit, lambda);
end
