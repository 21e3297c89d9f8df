function [x, error_norm, residual_norm, niters] = hybrid_ab_gmres_rtp(A, B, b, x_true, tol, maxit, lambda)
% Signature of the reference's hybrid_ab_gmres_rtp.m:1; the solve runs on the MI355X
% (hgm_hybrid_ab_gmres_rtp through hgmres_mex).  Histories come back as 1:niters.
[x, error_norm, residual_norm, niters] = hgmres_mex('hybrid_ab_gmres_rtp', A, B, b, x_true, tol, maxit, lambda);
end
