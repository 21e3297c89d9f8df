function [x, err, res, niters, phi_final, dphi_final, phi_iter, dphi_iter] = ABgmres_nonhybrid_bounds( ...
    A, B, b, x_true, tol, maxit, DeltaM)
% Signature of the reference's ABgmres_nonhybrid_bounds.m:1-2.  Outputs 1-4 are the device
% solve (hgm_gmres_bounds); outputs 5-8 (filter factors and their perturbation) come from
% hgm_gmres_bounds_filter, where eig(M) is replaced by device Ritz pairs of M.  DeltaM may be
% the formed product or, at scale, a cell {L, R} with DeltaM = L*R (never formed).
if nargout <= 4
    [x, err, res, niters] = hgmres_mex('gmres_bounds', 'ab', 0, A, B, b, x_true, tol, maxit, 0);
    return
end
if iscell(DeltaM)
    L = DeltaM{1}; R = DeltaM{2};
else
    L = DeltaM; R = [];
end
[x, err, res, niters, phi_final, dphi_final, phi_iter, dphi_iter] = hgmres_mex('gmres_bounds', 'ab', 0, A, B, b, x_true, tol, maxit, 0, L, R);
end
