function [x, error_norm, residual_norm, niters] = hybrid_ba_gmres_rtp(A, B, b, x_true, tol, maxit, lambda)
% Signature of the reference's hybrid_ba_gmres_rtp.m:1 (hgm_hybrid_ba_gmres_rtp on the MI355X).
[x, error_norm, residual_norm, niters] = hgmres_mex('hybrid_ba_gmres_rtp', A, B, b, x_true, tol, maxit, lambda);
end
