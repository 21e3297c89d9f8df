/*
 * hgmres_mex.c -- MATLAB gateway of libhgmres (the reference-side binding of include/hgmres.h).
 *
 * The reference (luisayang-malaxiangguo/Hybrid-GMRES) is pure MATLAB with no FFI.  Its solver
 * functions keep their signatures: the wrapper .m files in matlab/ replace the
 * bodies of the reference's solver .m files with one call into this gateway, which forwards to
 * the C ABI on the MI355X.  Every entry point of the ABI that a reference .m function maps to is
 * dispatched here:
 *
 *   hgmres_mex('hybrid_ab_gmres_rtp', A,B,b,x_true,tol,maxit,lambda)  hybrid_ab_gmres_rtp.m:1
 *   hgmres_mex('hybrid_ba_gmres_rtp', A,B,b,x_true,tol,maxit,lambda)  hybrid_ba_gmres_rtp.m:1
 *   hgmres_mex('lsqr_solver', A,b,x_true,tol,maxit)                   lsqr_solver.m:1
 *   hgmres_mex('lsmr_solver', A,b,x_true,tol,maxit)                   lsmr_solver.m:1 (x_true may be [])
 *   hgmres_mex('hybrid_lsqr_solver', A,b,x_true,tol,maxit,lambda)     hybrid_lsqr_solver.m:1
 *   hgmres_mex('hybrid_lsmr_solver', A,b,x_true,tol,maxit,lambda)     hybrid_lsmr_solver.m:1
 *   hgmres_mex('gcv_function', lambda,A,B,b,m,k_gcv,gcv_type)         gcv_function.m:1
 *   hgmres_mex('arnoldi', A,B,b,k,gcv_type)      -> [H, beta, kdone]  gcv_function.m:3-33 (cached H)
 *   hgmres_mex('gcv_fminbnd', H,beta,trace_m,lo,hi,tolx) -> [lambda, gcv]   analyze_regularization.m:37-46
 *   hgmres_mex('gmres_bounds', side,hybrid, A,B,b,x_true,tol,maxit,lambda, DeltaM[, DeltaR[, ritz_steps]])
 *        -> [x,err,res,niters,phi_final,dphi_final,phi_iter,dphi_iter]   {AB,BA}gmres_{hybrid,nonhybrid}_bounds.m:1-2
 *   hgmres_mex('device', d)                      select the HIP device (default 0)
 *   hgmres_mex('parity', 'auto'|'on'|'off')      summation orders (below; default 'auto')
 *
 * Summation orders.  MATLAB's own orders (MKL-blocked dot products, its sparse mtimes) cannot be
 * reproduced; libhgmres' fixed-order parity mode (HGM_OPT_PARITY) runs the
 * reference's sequence of operations in one documented order, in which it is bit-identical to the
 * oracle restatement.  'auto' (the default) selects it for every problem the reference itself runs
 * -- operators of at most HGM_PARITY_AUTO_DIM = 4096 rows and columns (the n = 32 shaw/heat/deriv2
 * drivers, the 32 x 32 phantom of run_2D_phantom.m) -- so gcv_function.m / analyze_regularization.m
 * see oracle-identical outputs there without opting in, and the production kernels (fused,
 * reordered sums) above it.  'on' / 'off' force one or the other.  NOTE: 'auto' changed the
 * default in round 4 -- callers at <= 4096 x 4096 now get the fixed-order kernels unless they set
 * 'off'.  The option is set per call from that call's operator on the gateway's private context
 * (g_ctx), so no choice outlives its call.
 *
 * Operands: MATLAB sparse (CSC, 64-bit mwIndex) is handed over as is (hgm_mat_create_csc); a
 * dense double matrix (the n = 32 drivers' shaw/deriv2 operators) is handed over as a CSC that
 * stores every entry.  Histories are allocated maxit long and truncated to 1:niters
 * (hybrid_ab_gmres_rtp.m:41-43, lsmr_solver.m:79-82).  A breakdown at k = 1, where the reference
 * never assigns x, raises MATLAB's own 'Output argument "x" not assigned' error.
 *
 * Build (needs MATLAB, absent from this image; tests/mexmock exercises the same source against a
 * stand-in of the mx API):
 *   mex -R2018a hgmres_mex.c -I<repo>/include -L<repo>/hybrid-gmres_amd/hgmres -lhgmres
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>

#include "hgmres.h"
#include "mex.h"

static hgm_ctx* g_ctx = NULL;
static int g_device = 0;

#define HGM_PARITY_AUTO_DIM 4096
static int g_parity = -1;   /* -1 auto, 0 off, 1 on */

/* operators created during one call, destroyed before returning or raising */
#define MAX_OPS 8
static hgm_mat* g_ops[MAX_OPS];
static int g_nops = 0;

static void release_ops(void) {
    for (int i = 0; i < g_nops; ++i) hgm_mat_destroy(g_ops[i]);
    g_nops = 0;
}

static void at_exit(void) {
    release_ops();
    if (g_ctx) hgm_ctx_destroy(g_ctx);
    g_ctx = NULL;
}

static void fail(const char* id, const char* msg) {
    release_ops();
    mexErrMsgIdAndTxt(id, "%s", msg);
}

static void check(int st) {
    if (st == HGM_OK) return;
    if (st == HGM_E_NOT_ASSIGNED)
        fail("MATLAB:unassignedOutputs", "Output argument \"x\" (and possibly others) not assigned during call.");
    fail("hgmres:solve", g_ctx ? hgm_last_error(g_ctx) : "libhgmres error");
}

static hgm_ctx* ctx(void) {
    if (!g_ctx) {
        if (hgm_ctx_create(g_device, &g_ctx) != HGM_OK || !g_ctx) {
            g_ctx = NULL;
            fail("hgmres:device", "hgmres: no usable HIP device (libhgmres needs an MI355X)");
        }
        mexAtExit(at_exit);
    }
    return g_ctx;
}

static void need_double(const mxArray* a, const char* what) {
    if (!mxIsDouble(a) || mxIsComplex(a)) {
        char msg[160];
        snprintf(msg, sizeof msg, "hgmres: %s must be a real double array", what);
        fail("hgmres:arg", msg);
    }
}

static double scalar(const mxArray* a, const char* what) {
    need_double(a, what);
    if (mxGetNumberOfElements(a) != 1) {
        char msg[160];
        snprintf(msg, sizeof msg, "hgmres: %s must be a scalar", what);
        fail("hgmres:arg", msg);
    }
    return mxGetScalar(a);
}

/* a column vector of exactly len doubles (NULL for [] when allow_empty) */
static const double* vec(const mxArray* a, int64_t len, const char* what, int allow_empty) {
    if (allow_empty && mxIsEmpty(a)) return NULL;
    need_double(a, what);
    if (mxIsSparse(a) || (int64_t)mxGetNumberOfElements(a) != len) {
        char msg[160];
        snprintf(msg, sizeof msg, "hgmres: %s must be a dense vector of length %lld", what, (long long)len);
        fail("hgmres:arg", msg);
    }
    return mxGetDoubles(a);
}

/* MATLAB operand -> device operator (sparse CSC as is; dense as a CSC of every entry) */
static hgm_mat* op(const mxArray* a, const char* what) {
    need_double(a, what);
    if (g_nops >= MAX_OPS) fail("hgmres:internal", "hgmres: too many operands");
    const int64_t m = (int64_t)mxGetM(a), n = (int64_t)mxGetN(a);
    hgm_mat* M = NULL;
    int st;
    if (mxIsSparse(a)) {
        const mwIndex* jc = mxGetJc(a);
        st = hgm_mat_create_csc(ctx(), m, n, (int64_t)jc[n], (const int64_t*)jc, (const int64_t*)mxGetIr(a),
                                mxGetDoubles(a), HGM_F64, &M);
    } else {
        int64_t* jc = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
        int64_t* ir = (int64_t*)malloc(sizeof(int64_t) * (size_t)(m * n > 0 ? m * n : 1));
        if (!jc || !ir) {
            free(jc);
            free(ir);
            fail("hgmres:nomem", "hgmres: out of host memory");
        }
        for (int64_t j = 0; j <= n; ++j) jc[j] = j * m;
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i < m; ++i) ir[j * m + i] = i;
        st = hgm_mat_create_csc(ctx(), m, n, m * n, jc, ir, mxGetDoubles(a), HGM_F64, &M);
        free(jc);
        free(ir);
    }
    check(st);
    g_ops[g_nops++] = M;
    return M;
}

/* the summation orders for a solve on operator A (see the header: 'auto' = parity mode for
 * reference-size operators) */
static void parity_for(const hgm_mat* A) {
    int64_t m = 0, n = 0;
    hgm_mat_info(A, &m, &n, NULL, NULL);
    const int on = g_parity >= 0 ? g_parity : (m <= HGM_PARITY_AUTO_DIM && n <= HGM_PARITY_AUTO_DIM);
    check(hgm_ctx_set_option(ctx(), HGM_OPT_PARITY, on ? 1.0 : 0.0));
}

static hgm_mat* transpose_op(hgm_mat* A) {
    hgm_mat* T = NULL;
    check(hgm_mat_transpose(ctx(), A, &T));
    g_ops[g_nops++] = T;
    return T;
}

static int side_of(const mxArray* a) {
    char s[8];
    if (!mxIsChar(a) || mxGetString(a, s, sizeof s) != 0) fail("hgmres:arg", "hgmres: gcv_type/side must be 'ab' or 'ba'");
    if (!strcmp(s, "ab") || !strcmp(s, "AB")) return HGM_SIDE_AB;
    if (!strcmp(s, "ba") || !strcmp(s, "BA")) return HGM_SIDE_BA;
    fail("hgmres:arg", "hgmres: gcv_type/side must be 'ab' or 'ba'");
    return -1;
}

static int maxit_of(const mxArray* a) {
    const double v = scalar(a, "maxit");
    if (!(v >= 1) || v != (double)(int)v) fail("hgmres:arg", "hgmres: maxit must be a positive integer");
    return (int)v;
}

static mxArray* column(const double* v, int len) {
    mxArray* r = mxCreateDoubleMatrix((mwSize)len, 1, mxREAL);
    if (len > 0) memcpy(mxGetDoubles(r), v, sizeof(double) * (size_t)len);
    return r;
}

static void nargs(int nrhs, int lo, int hi, const char* fn) {
    if (nrhs - 1 < lo || nrhs - 1 > hi) {
        char msg[160];
        snprintf(msg, sizeof msg, "hgmres: wrong number of arguments for %s", fn);
        fail("hgmres:nargin", msg);
    }
}

/* [x, error_norm, residual_norm, niters] of the GMRES-family solvers */
static void gmres_rtp(int nlhs, mxArray* plhs[], const mxArray* prhs[], int ba) {
    hgm_mat* A = op(prhs[1], "A");
    parity_for(A);
    hgm_mat* B = op(prhs[2], "B");
    int64_t m = 0, n = 0;
    hgm_mat_info(A, &m, &n, NULL, NULL);
    const double* b = vec(prhs[3], m, "b", 0);
    const double* xt = vec(prhs[4], n, "x_true", 0);
    const double tol = scalar(prhs[5], "tol");
    const int maxit = maxit_of(prhs[6]);
    const double lambda = scalar(prhs[7], "lambda");
    mxArray* x = mxCreateDoubleMatrix((mwSize)n, 1, mxREAL);
    mxArray* e = mxCreateDoubleMatrix((mwSize)maxit, 1, mxREAL);
    mxArray* r = mxCreateDoubleMatrix((mwSize)maxit, 1, mxREAL);
    int k = 0;
    check((ba ? hgm_hybrid_ba_gmres_rtp : hgm_hybrid_ab_gmres_rtp)(ctx(), A, B, b, xt, tol, maxit, lambda,
                                                                    mxGetDoubles(x), mxGetDoubles(e),
                                                                    mxGetDoubles(r), &k));
    mxSetM(e, (mwSize)k);                             /* error_norm(1:niters)    :41-43 */
    mxSetM(r, (mwSize)k);                             /* residual_norm(1:niters) */
    plhs[0] = x;
    if (nlhs > 1) plhs[1] = e;
    if (nlhs > 2) plhs[2] = r;
    if (nlhs > 3) plhs[3] = mxCreateDoubleScalar(k);
}

/* lsqr_solver / hybrid_lsqr_solver / hybrid_lsmr_solver: [x, error_norm, residual_norm, niters] */
static void gkb(int nlhs, mxArray* plhs[], const mxArray* prhs[], int which /* 0 lsqr, 1 hlsqr, 2 hlsmr */) {
    hgm_mat* A = op(prhs[1], "A");
    parity_for(A);
    hgm_mat* At = transpose_op(A);
    int64_t m = 0, n = 0;
    hgm_mat_info(A, &m, &n, NULL, NULL);
    const double* b = vec(prhs[2], m, "b", 0);
    const double* xt = vec(prhs[3], n, "x_true", 0);
    const double tol = scalar(prhs[4], "tol");
    const int maxit = maxit_of(prhs[5]);
    const double lambda = which ? scalar(prhs[6], "lambda") : 0.0;
    mxArray* x = mxCreateDoubleMatrix((mwSize)n, 1, mxREAL);
    mxArray* e = mxCreateDoubleMatrix((mwSize)maxit, 1, mxREAL);
    mxArray* r = mxCreateDoubleMatrix((mwSize)maxit, 1, mxREAL);
    int k = 0;
    if (which == 0)
        check(hgm_lsqr_solver(ctx(), A, At, b, xt, tol, maxit, mxGetDoubles(x), mxGetDoubles(e), mxGetDoubles(r), &k));
    else if (which == 1)
        check(hgm_hybrid_lsqr_solver(ctx(), A, At, b, xt, tol, maxit, lambda, mxGetDoubles(x), mxGetDoubles(e),
                                     mxGetDoubles(r), &k));
    else
        check(hgm_hybrid_lsmr_solver(ctx(), A, At, b, xt, tol, maxit, lambda, mxGetDoubles(x), mxGetDoubles(e),
                                     mxGetDoubles(r), &k));
    mxSetM(e, (mwSize)k);
    mxSetM(r, (mwSize)k);
    plhs[0] = x;
    if (nlhs > 1) plhs[1] = e;
    if (nlhs > 2) plhs[2] = r;
    if (nlhs > 3) plhs[3] = mxCreateDoubleScalar(k);
}

/* lsmr_solver: [x, err_hist, res_hist, ar_hist, iters]; the .m wrapper applies the defaults of
 * lsmr_solver.m:3,5 (tol = 1e-6, maxit = min(m,n)) */
static void lsmr(int nlhs, mxArray* plhs[], const mxArray* prhs[]) {
    hgm_mat* A = op(prhs[1], "A");
    parity_for(A);
    hgm_mat* At = transpose_op(A);
    int64_t m = 0, n = 0;
    hgm_mat_info(A, &m, &n, NULL, NULL);
    const double* b = vec(prhs[2], m, "b", 0);
    const double* xt = vec(prhs[3], n, "x_true", 1);
    const double tol = scalar(prhs[4], "tol");
    const int maxit = maxit_of(prhs[5]);
    mxArray* x = mxCreateDoubleMatrix((mwSize)n, 1, mxREAL);
    mxArray* eh = mxCreateDoubleMatrix((mwSize)maxit, 1, mxREAL);
    mxArray* rh = mxCreateDoubleMatrix((mwSize)maxit, 1, mxREAL);
    mxArray* ah = mxCreateDoubleMatrix((mwSize)maxit, 1, mxREAL);
    int k = 0;
    check(hgm_lsmr_solver(ctx(), A, At, b, xt, tol, maxit, mxGetDoubles(x), mxGetDoubles(eh), mxGetDoubles(rh),
                          mxGetDoubles(ah), &k));
    mxSetM(eh, (mwSize)k);                            /* lsmr_solver.m:79-82 */
    mxSetM(rh, (mwSize)k);
    mxSetM(ah, (mwSize)k);
    plhs[0] = x;
    if (nlhs > 1) plhs[1] = eh;
    if (nlhs > 2) plhs[2] = rh;
    if (nlhs > 3) plhs[3] = ah;
    if (nlhs > 4) plhs[4] = mxCreateDoubleScalar(k);
}

/* gcv_val = gcv_function(lambda, A, B, b, m, k_gcv, gcv_type) */
static void gcv(mxArray* plhs[], const mxArray* prhs[]) {
    const double lambda = scalar(prhs[1], "lambda");
    hgm_mat* A = op(prhs[2], "A");
    parity_for(A);
    hgm_mat* B = op(prhs[3], "B");
    int64_t m = 0, n = 0;
    hgm_mat_info(A, &m, &n, NULL, NULL);
    const double* b = vec(prhs[4], m, "b", 0);
    const double mm = scalar(prhs[5], "m");
    const double kg = scalar(prhs[6], "k_gcv");
    if (!(kg >= 1) || kg != (double)(int)kg) fail("hgmres:arg", "hgmres: k_gcv must be a positive integer");
    const int side = side_of(prhs[7]);
    double g = 0;
    check(hgm_gcv_function(ctx(), lambda, A, B, b, (int64_t)mm, (int)kg, side, &g));
    plhs[0] = mxCreateDoubleScalar(g);
}

/* [H, beta, kdone] = hgmres_mex('arnoldi', A, B, b, k, gcv_type) */
static void arnoldi(int nlhs, mxArray* plhs[], const mxArray* prhs[]) {
    hgm_mat* A = op(prhs[1], "A");
    parity_for(A);
    hgm_mat* B = op(prhs[2], "B");
    int64_t m = 0, n = 0;
    hgm_mat_info(A, &m, &n, NULL, NULL);
    const double* b = vec(prhs[3], m, "b", 0);
    const int k = maxit_of(prhs[4]);
    const int side = side_of(prhs[5]);
    mxArray* H = mxCreateDoubleMatrix((mwSize)(k + 1), (mwSize)k, mxREAL);
    double beta = 0;
    int kd = 0;
    check(hgm_arnoldi(ctx(), A, B, b, k, side, 1e-12, HGM_MGS, mxGetDoubles(H), &beta, &kd));
    plhs[0] = H;
    if (nlhs > 1) plhs[1] = mxCreateDoubleScalar(beta);
    if (nlhs > 2) plhs[2] = mxCreateDoubleScalar(kd);
}

/* [lambda, gcv] = hgmres_mex('gcv_fminbnd', H, beta, trace_m, lo, hi, tolx)  (host only) */
static void gcv_fminbnd(int nlhs, mxArray* plhs[], const mxArray* prhs[]) {
    need_double(prhs[1], "H");
    const int k = (int)mxGetN(prhs[1]);
    if (k < 1 || (int)mxGetM(prhs[1]) != k + 1 || mxIsSparse(prhs[1]))
        fail("hgmres:arg", "hgmres: H must be a dense (k+1) x k matrix");
    double lam = 0, g = 0;
    const int st = hgm_gcv_fminbnd(mxGetDoubles(prhs[1]), k, scalar(prhs[2], "beta"), scalar(prhs[3], "trace_m"),
                                   scalar(prhs[4], "lo"), scalar(prhs[5], "hi"), scalar(prhs[6], "tolx"), &lam, &g);
    if (st != HGM_OK) fail("hgmres:arg", "hgmres: invalid fminbnd arguments");
    plhs[0] = mxCreateDoubleScalar(lam);
    if (nlhs > 1) plhs[1] = mxCreateDoubleScalar(g);
}

/* the 8 outputs of {AB,BA}gmres_{hybrid,nonhybrid}_bounds */
static void bounds(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nlhs > 4 && (nrhs <= 10 || mxIsEmpty(prhs[10]))) fail("hgmres:nargout", "hgmres: outputs 5-8 need DeltaM");
    const int side = side_of(prhs[1]);
    const int hybrid = scalar(prhs[2], "hybrid") != 0.0;
    hgm_mat* A = op(prhs[3], "A");
    parity_for(A);
    hgm_mat* B = op(prhs[4], "B");
    int64_t m = 0, n = 0;
    hgm_mat_info(A, &m, &n, NULL, NULL);
    const double* b = vec(prhs[5], m, "b", 0);
    const double* xt = vec(prhs[6], n, "x_true", 0);
    const double tol = scalar(prhs[7], "tol");
    const int maxit = maxit_of(prhs[8]);
    const double lambda = scalar(prhs[9], "lambda");
    const int want_phi = nlhs > 4 && nrhs > 10 && !mxIsEmpty(prhs[10]);
    mxArray* x = mxCreateDoubleMatrix((mwSize)n, 1, mxREAL);
    mxArray* e = mxCreateDoubleMatrix((mwSize)maxit, 1, mxREAL);
    mxArray* r = mxCreateDoubleMatrix((mwSize)maxit, 1, mxREAL);
    int k = 0;
    if (!want_phi) {
        check(hgm_gmres_bounds(ctx(), A, B, b, xt, tol, maxit, lambda, side, hybrid, mxGetDoubles(x),
                               mxGetDoubles(e), mxGetDoubles(r), &k));
    } else {
        hgm_mat* DL = op(prhs[10], "DeltaM");
        hgm_mat* DR = (nrhs > 11 && !mxIsEmpty(prhs[11])) ? op(prhs[11], "DeltaM factor") : NULL;
        const int ritz = nrhs > 12 ? (int)scalar(prhs[12], "ritz_steps") : 0;
        double* phi = (double*)mxCalloc((size_t)maxit * maxit, sizeof(double));
        double* dphi = (double*)mxCalloc((size_t)maxit * maxit, sizeof(double));
        double* Hk = (double*)mxCalloc((size_t)(maxit + 1) * maxit, sizeof(double));
        double* mu = (double*)mxCalloc((size_t)maxit, sizeof(double));
        double* rres = (double*)mxCalloc((size_t)maxit, sizeof(double));
        hgm_opts o = {0, HGM_MGS, Hk};
        check(hgm_gmres_bounds_filter(ctx(), &o, A, B, b, xt, tol, maxit, lambda, side, hybrid, DL, DR, ritz,
                                      mxGetDoubles(x), mxGetDoubles(e), mxGetDoubles(r), &k, phi, dphi, mu, rres));
        /* a breakdown at iteration k (H(k+1,k) == 0, *_bounds.m:31 breaks before :80) leaves
           phi_iter{k} unassigned in the reference: that cell alone is [] here; every other cell
           holds its j values, NaN included (e.g. b = 0 gives NaN vectors, as MATLAB does) */
        const int broke = k >= 1 && Hk[(size_t)(k - 1) * (maxit + 1) + k] == 0.0;
        const int kf = broke ? k - 1 : k;
        /* eig(M) of *_bounds.m:4-9 is replaced by Ritz pairs: exact for ritz_steps = dim (the default
           for dim <= 1024), otherwise approximations whose residuals are reported here */
        double rmax = 0, mu1 = kf > 0 ? fabs(mu[0]) : 0;
        for (int j = 0; j < kf; ++j) rmax = rres[j] > rmax ? rres[j] : rmax;
        if (kf > 0 && !(rmax <= 1e-8 * mu1))
            mexWarnMsgIdAndTxt("hgmres:ritz", "hgmres: the %d leading Ritz values stand in for eig(M) with a "
                               "relative residual of %.2e; pass ritz_steps = size(M,1) for eig(M) itself", kf,
                               mu1 > 0 ? rmax / mu1 : rmax);
        mxArray* pc = mxCreateCellMatrix((mwSize)k, 1);
        mxArray* dc = mxCreateCellMatrix((mwSize)k, 1);
        for (int j = 1; j <= k; ++j) {
            const int len = (broke && j == k) ? 0 : j;
            mxSetCell(pc, (mwIndex)(j - 1), column(phi + (size_t)(j - 1) * maxit, len));
            mxSetCell(dc, (mwIndex)(j - 1), column(dphi + (size_t)(j - 1) * maxit, len));
        }
        const int lk = broke ? 0 : k;
        plhs[4] = column(phi + (size_t)(k - 1) * maxit, lk);               /* phi_final  = phi_iter{k} */
        if (nlhs > 5) plhs[5] = column(dphi + (size_t)(k - 1) * maxit, lk); /* dphi_final */
        if (nlhs > 6) plhs[6] = pc;
        if (nlhs > 7) plhs[7] = dc;
        mxFree(Hk);
        mxFree(mu);
        mxFree(rres);
        mxFree(phi);
        mxFree(dphi);
    }
    mxSetM(e, (mwSize)k);
    mxSetM(r, (mwSize)k);
    plhs[0] = x;
    if (nlhs > 1) plhs[1] = e;
    if (nlhs > 2) plhs[2] = r;
    if (nlhs > 3) plhs[3] = mxCreateDoubleScalar(k);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char fn[32];
    if (nrhs < 1 || !mxIsChar(prhs[0]) || mxGetString(prhs[0], fn, sizeof fn) != 0)
        fail("hgmres:nargin", "hgmres: the first argument names the function");
    if (!strcmp(fn, "hybrid_ab_gmres_rtp") || !strcmp(fn, "hybrid_ba_gmres_rtp")) {
        nargs(nrhs, 7, 7, fn);
        gmres_rtp(nlhs, plhs, prhs, fn[7] == 'b');
    } else if (!strcmp(fn, "lsqr_solver")) {
        nargs(nrhs, 5, 5, fn);
        gkb(nlhs, plhs, prhs, 0);
    } else if (!strcmp(fn, "hybrid_lsqr_solver")) {
        nargs(nrhs, 6, 6, fn);
        gkb(nlhs, plhs, prhs, 1);
    } else if (!strcmp(fn, "hybrid_lsmr_solver")) {
        nargs(nrhs, 6, 6, fn);
        gkb(nlhs, plhs, prhs, 2);
    } else if (!strcmp(fn, "lsmr_solver")) {
        nargs(nrhs, 5, 5, fn);
        lsmr(nlhs, plhs, prhs);
    } else if (!strcmp(fn, "gcv_function")) {
        nargs(nrhs, 7, 7, fn);
        gcv(plhs, prhs);
    } else if (!strcmp(fn, "arnoldi")) {
        nargs(nrhs, 5, 5, fn);
        arnoldi(nlhs, plhs, prhs);
    } else if (!strcmp(fn, "gcv_fminbnd")) {
        nargs(nrhs, 6, 6, fn);
        gcv_fminbnd(nlhs, plhs, prhs);
    } else if (!strcmp(fn, "gmres_bounds")) {
        nargs(nrhs, 9, 12, fn);
        bounds(nlhs, plhs, nrhs, prhs);
    } else if (!strcmp(fn, "parity")) {
        nargs(nrhs, 1, 1, fn);
        char mode[8];
        if (!mxIsChar(prhs[1]) || mxGetString(prhs[1], mode, sizeof mode) != 0)
            fail("hgmres:arg", "hgmres: parity mode is 'auto', 'on' or 'off'");
        if (!strcmp(mode, "auto")) g_parity = -1;
        else if (!strcmp(mode, "on")) g_parity = 1;
        else if (!strcmp(mode, "off")) g_parity = 0;
        else fail("hgmres:arg", "hgmres: parity mode is 'auto', 'on' or 'off'");
    } else if (!strcmp(fn, "device")) {
        nargs(nrhs, 1, 1, fn);
        const double d = scalar(prhs[1], "device");
        if (g_ctx) at_exit();
        g_device = (int)d;
    } else {
        fail("hgmres:unknown", "hgmres: unknown function");
    }
    release_ops();
}
