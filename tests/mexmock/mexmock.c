/* TEST INFRASTRUCTURE -- implementation of the mx API stand-in (see mex.h) and the entry points
 * tests/test_mex_gateway.py calls through ctypes. */
#define _POSIX_C_SOURCE 200809L
#include <setjmp.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

enum { C_DOUBLE = 0, C_CHAR = 1, C_CELL = 2 };

struct mxArray_tag {
    int cls;
    int sparse;
    size_t m, n;
    double* pr;
    mwIndex* jc;
    mwIndex* ir;
    char* str;
    mxArray** cells;
};

mwSize mxGetM(const mxArray* a) { return a->m; }
mwSize mxGetN(const mxArray* a) { return a->n; }
size_t mxGetNumberOfElements(const mxArray* a) { return a->m * a->n; }
int mxIsDouble(const mxArray* a) { return a->cls == C_DOUBLE; }
int mxIsComplex(const mxArray* a) { (void)a; return 0; }
int mxIsSparse(const mxArray* a) { return a->sparse; }
int mxIsChar(const mxArray* a) { return a->cls == C_CHAR; }
int mxIsCell(const mxArray* a) { return a->cls == C_CELL; }
int mxIsEmpty(const mxArray* a) { return a->m == 0 || a->n == 0; }
int mxGetString(const mxArray* a, char* buf, mwSize len) {
    if (a->cls != C_CHAR || len == 0) return 1;
    const size_t l = strlen(a->str);
    strncpy(buf, a->str, len - 1);
    buf[len - 1] = 0;
    return l >= len;
}
double mxGetScalar(const mxArray* a) { return (a->cls == C_DOUBLE && a->pr && a->m > 0 && a->n > 0) ? a->pr[0] : 0.0; }
double* mxGetDoubles(const mxArray* a) { return a->cls == C_DOUBLE ? a->pr : NULL; }
mwIndex* mxGetJc(const mxArray* a) { return a->jc; }
mwIndex* mxGetIr(const mxArray* a) { return a->ir; }

mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) {
    (void)c;
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->cls = C_DOUBLE;
    a->m = m;
    a->n = n;
    a->pr = (double*)calloc(m * n > 0 ? m * n : 1, sizeof(double));
    return a;
}
mxArray* mxCreateDoubleScalar(double v) {
    mxArray* a = mxCreateDoubleMatrix(1, 1, mxREAL);
    a->pr[0] = v;
    return a;
}
void mxSetM(mxArray* a, mwSize m) { a->m = m; }
mxArray* mxCreateCellMatrix(mwSize m, mwSize n) {
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->cls = C_CELL;
    a->m = m;
    a->n = n;
    a->cells = (mxArray**)calloc(m * n > 0 ? m * n : 1, sizeof(mxArray*));
    return a;
}
void mxSetCell(mxArray* a, mwIndex i, mxArray* v) { a->cells[i] = v; }
mxArray* mxGetCell(const mxArray* a, mwIndex i) { return a->cells[i]; }
void* mxCalloc(size_t n, size_t size) { return calloc(n, size); }
void mxFree(void* p) { free(p); }
void mxDestroyArray(mxArray* a) {
    if (!a) return;
    if (a->cls == C_CELL)
        for (size_t i = 0; i < a->m * a->n; ++i) mxDestroyArray(a->cells[i]);
    free(a->pr);
    free(a->jc);
    free(a->ir);
    free(a->str);
    free(a->cells);
    free(a);
}

static jmp_buf g_jmp;
static char g_id[128], g_msg[512];
static void (*g_exit)(void) = NULL;

void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
    snprintf(g_id, sizeof g_id, "%s", id);
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_msg, sizeof g_msg, fmt, ap);
    va_end(ap);
    longjmp(g_jmp, 1);
}
/* warnings: the last one is kept (mock_last_warning) */
static char g_wid[128], g_wmsg[1024];
static int g_nwarn;
void mexWarnMsgIdAndTxt(const char* id, const char* fmt, ...) {
    snprintf(g_wid, sizeof g_wid, "%s", id);
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_wmsg, sizeof g_wmsg, fmt, ap);
    va_end(ap);
    ++g_nwarn;
}
int mock_last_warning(char* id, char* msg, int len) {
    snprintf(id, len, "%s", g_wid);
    snprintf(msg, len, "%s", g_wmsg);
    const int n = g_nwarn;
    g_nwarn = 0;
    g_wid[0] = g_wmsg[0] = 0;
    return n;
}
int mexAtExit(void (*fn)(void)) {
    g_exit = fn;
    return 0;
}

/* ---- test-facing entry points ---- */
mxArray* mock_double(size_t m, size_t n, const double* data) {
    mxArray* a = mxCreateDoubleMatrix(m, n, mxREAL);
    if (data && m > 0 && n > 0) memcpy(a->pr, data, sizeof(double) * m * n);
    return a;
}
mxArray* mock_sparse(size_t m, size_t n, size_t nnz, const int64_t* jc, const int64_t* ir, const double* pr) {
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->cls = C_DOUBLE;
    a->sparse = 1;
    a->m = m;
    a->n = n;
    a->jc = (mwIndex*)malloc(sizeof(mwIndex) * (n + 1));
    a->ir = (mwIndex*)malloc(sizeof(mwIndex) * (nnz ? nnz : 1));
    a->pr = (double*)malloc(sizeof(double) * (nnz ? nnz : 1));
    for (size_t j = 0; j <= n; ++j) a->jc[j] = (mwIndex)jc[j];
    for (size_t i = 0; i < nnz; ++i) {
        a->ir[i] = (mwIndex)ir[i];
        a->pr[i] = pr[i];
    }
    return a;
}
mxArray* mock_string(const char* s) {
    mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
    a->cls = C_CHAR;
    a->m = 1;
    a->n = strlen(s);
    a->str = strdup(s);
    return a;
}
/* 0: ok; 1: mexErrMsgIdAndTxt raised (id / message copied out) */
int mock_call(int nlhs, mxArray** plhs, int nrhs, const mxArray** prhs, char* id, char* msg, int len) {
    for (int i = 0; i < nlhs; ++i) plhs[i] = NULL;
    if (setjmp(g_jmp)) {
        snprintf(id, len, "%s", g_id);
        snprintf(msg, len, "%s", g_msg);
        return 1;
    }
    mexFunction(nlhs, plhs, nrhs, prhs);
    return 0;
}
void mock_exit(void) {
    if (g_exit) g_exit();
    g_exit = NULL;
}
