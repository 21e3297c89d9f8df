function gcv_val = gcv_function(lambda, A, B, b, m, k_gcv, gcv_type)
% Signature of the reference's gcv_function.m:1 (hgm_gcv_function: the k_gcv-step Arnoldi on the
% MI355X, the lambda-dependent part on the host).  For an fminbnd loop over lambda, call
%   [H, beta] = hgmres_mex('arnoldi', A, B, b, k_gcv, gcv_type);
%   lambda = hgmres_mex('gcv_fminbnd', H, beta, trace_m, lo, hi, tolx);
% once instead: the values equal this function's at every lambda.
gcv_val = hgmres_mex('gcv_function', lambda, A, B, b, m, k_gcv, gcv_type);
end
