function [x, error_norm, residual_norm, niters] = hybrid_lsqr_solver(A, b, x_true, tol, maxit, lambda)
% Signature of the reference's hybrid_lsqr_solver.m:1: LSQR on [A; sqrt(lambda) I] with the
% augmentation kept implicit on the device (hgm_hybrid_lsqr_solver).
[x, error_norm, residual_norm, niters] = hgmres_mex('hybrid_lsqr_solver', A, b, x_true, tol, maxit, lambda);
end
