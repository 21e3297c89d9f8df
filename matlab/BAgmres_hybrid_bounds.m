function [x, error_norm, residual_norm, niters, phi_final, dphi_final, phi_iter, dphi_iter] = BAgmres_hybrid_bounds( ...
    A, B, b, x_true, tol, maxit, lambda, DeltaM)
% Signature of the reference's BAgmres_hybrid_bounds.m:1-2.  Outputs 1-4 are the device
% solve (hgm_gmres_bounds); outputs 5-8 (filter factors and their perturbation) come from
% hgm_gmres_bounds_filter, where eig(M) is replaced by device Ritz pairs of M.  DeltaM may be
% the formed product or, at scale, a cell {L, R} with DeltaM = L*R (never formed).
if nargout <= 4
    [x, error_norm, residual_norm, niters] = hgmres_mex('gmres_bounds', 'ba', 1, A, B, b, x_true, tol, maxit, lambda);
    return
end
if iscell(DeltaM)
    L = DeltaM{1}; R = DeltaM{2};
else
    L = DeltaM; R = [];
end
[x, error_norm, residual_norm, niters, phi_final, dphi_final, phi_iter, dphi_iter] = hgmres_mex('gmres_bounds', 'ba', 1, A, B, b, x_true, tol, maxit, lambda, L, R);
end
