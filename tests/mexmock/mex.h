/*
 * TEST INFRASTRUCTURE -- a minimal stand-in for MATLAB's mex.h / matrix.h (the R2018a interleaved
 * mx API subset matlab/hgmres_mex.c uses), so the gateway source compiles and runs here without
 * MATLAB: tests/test_mex_gateway.py drives mexFunction through it and compares every dispatched
 * entry point with the Python binding.  Not a MATLAB substitute and not shipped.
 */
#ifndef HGM_MEXMOCK_H
#define HGM_MEXMOCK_H
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef size_t mwSize;
typedef size_t mwIndex;
typedef enum { mxREAL = 0, mxCOMPLEX = 1 } mxComplexity;
typedef struct mxArray_tag mxArray;

mwSize mxGetM(const mxArray* a);
mwSize mxGetN(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
int mxIsDouble(const mxArray* a);
int mxIsComplex(const mxArray* a);
int mxIsSparse(const mxArray* a);
int mxIsChar(const mxArray* a);
int mxIsCell(const mxArray* a);
int mxIsEmpty(const mxArray* a);
int mxGetString(const mxArray* a, char* buf, mwSize len);
double mxGetScalar(const mxArray* a);
double* mxGetDoubles(const mxArray* a);
mwIndex* mxGetJc(const mxArray* a);
mwIndex* mxGetIr(const mxArray* a);
mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray* mxCreateDoubleScalar(double v);
void mxSetM(mxArray* a, mwSize m);
mxArray* mxCreateCellMatrix(mwSize m, mwSize n);
void mxSetCell(mxArray* a, mwIndex i, mxArray* v);
mxArray* mxGetCell(const mxArray* a, mwIndex i);
void* mxCalloc(size_t n, size_t size);
void mxFree(void* p);
void mxDestroyArray(mxArray* a);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) __attribute__((noreturn));
void mexWarnMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexAtExit(void (*fn)(void));

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

#ifdef __cplusplus
}
#endif
#endif
