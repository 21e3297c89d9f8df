/*
 * ORACLE — all-core CPU SpMV for the bench's cpu_baseline leg (test infrastructure only;
 * never linked into libhgmres).
 *
 * y = M x for a CSR matrix, rows split into contiguous static blocks across OpenMP
 * threads.  Every row is summed sequentially in stored order with a separate multiply
 * and add (built with -ffp-contract=off), i.e. exactly scipy's csr_matvec
 * (`sum += Ax[jj] * Xx[Aj[jj]]`, scipy/sparse/sparsetools/csr.h), so the product is
 * bitwise identical to `M @ x` in oracle/restatement.py — only the wall time changes.
 * The reference computes these products with MATLAB's multithreaded sparse mtimes
 * (e.g. hybrid_ab_gmres_rtp.m:6,19; ABgmres_nonhybrid_bounds.m:25).
 */
#include <omp.h>
#include <stdint.h>

void oracle_csr_matvec(int64_t rows, const int64_t* rp, const int32_t* ci, const double* val, const double* x,
                       double* y) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < rows; ++i) {
        double s = 0.0;
        for (int64_t j = rp[i]; j < rp[i + 1]; ++j) s += val[j] * x[ci[j]];
        y[i] = s;
    }
}

/* fp32 (BASELINE configs[4]): the same sequential row sums in single precision, as scipy's
   csr_matvec<float> computes `A32 @ v32` (and libhgmres' parity-mode k_spmv_seq<float>). */
void oracle_csr_matvec_f32(int64_t rows, const int64_t* rp, const int32_t* ci, const float* val, const float* x,
                           float* y) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < rows; ++i) {
        float s = 0.0f;
        for (int64_t j = rp[i]; j < rp[i + 1]; ++j) s += val[j] * x[ci[j]];
        y[i] = s;
    }
}

/* fp32 in ANOTHER summation order (test infrastructure: the fp32 oracle's own rounding spread,
   tests/golden/make_golden.py dump_c5).  Row entries are visited forward (rev = 0) or backward
   (rev = 1) and dealt round-robin over `ways` accumulators (1..128), which are then combined by
   a pairwise tree -- the shape of a lane-parallel GPU row sum.  Each order is a correct fp32 sum
   of the same products; ways = 1, rev = 0 is oracle_csr_matvec_f32. */
void oracle_csr_matvec_f32_order(int64_t rows, const int64_t* rp, const int32_t* ci, const float* val,
                                 const float* x, float* y, int ways, int rev) {
    if (ways < 1) ways = 1;
    if (ways > 128) ways = 128;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < rows; ++i) {
        float acc[128];
        for (int w = 0; w < ways; ++w) acc[w] = 0.0f;
        const int64_t a = rp[i], len = rp[i + 1] - rp[i];
        for (int64_t t = 0; t < len; ++t) {
            const int64_t j = rev ? a + len - 1 - t : a + t;
            acc[t % ways] += val[j] * x[ci[j]];
        }
        for (int h = 1; h < ways; h *= 2)
            for (int w = 0; w + h < ways; w += 2 * h) acc[w] += acc[w + h];
        y[i] = acc[0];
    }
}

int oracle_num_threads(void) { return omp_get_max_threads(); }
