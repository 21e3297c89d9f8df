// HIP kernels of the Arnoldi/GMRES + Golub-Kahan inner loop other than SpMV (spmv.hip),
// written for gfx950 (CDNA4).
//
//  * MGS (hybrid_*_rtp.m:20-26): one launch per Gram-Schmidt pass j fusing
//    axpy_j (v -= h_j q_j) with the inner product of the NEXT column (q_{j+1}' v).  The
//    grid-wide sum of pass j's block partials is re-reduced, in a fixed order, by
//    every block of pass j+1 (identical bits in every block), so no separate reduce
//    launch and no host round trip is needed between passes.
//  * Reductions: per-lane sums -> wave butterfly -> 4-wave LDS sum in fixed order
//    (single 1024-thread launch for vectors up to 256 Ki entries).
//  * Krylov-basis GEMV (x = Q y) fused with the error monitor, elementwise GKB updates.
#include "device_common.h"

namespace hgm {

int parts_for(int64_t n) {
    // >= 2 element pairs per thread, up to MAX_PARTS blocks (256 CUs x 4)
    int64_t nb = (n + 2 * BS * 2 - 1) / (2 * BS * 2);
    if (nb < 1) nb = 1;
    if (nb > MAX_PARTS) nb = MAX_PARTS;
    return (int)nb;
}

// ------------------------------------------------------------------------------
// Reductions
// ------------------------------------------------------------------------------
template <typename T, int OP>   // 0: a.b   1: a.a   2: (a-b).(a-b)
__global__ __launch_bounds__(BS) void k_reduce_partial(int64_t n, const T* __restrict__ a,
                                                       const T* __restrict__ b,
                                                       T* __restrict__ parts) {
    __shared__ T sh[4];
    T acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
        if (OP == 0) acc += a[i] * b[i];
        else if (OP == 1) acc += a[i] * a[i];
        else { T d = a[i] - b[i]; acc += d * d; }
    }
    T tot = block_sum_all(acc, sh);
    if (threadIdx.x == 0) parts[blockIdx.x] = tot;
}

template <typename T>
__global__ __launch_bounds__(BS) void k_finalize(const T* __restrict__ parts, int np, T* out) {
    __shared__ T sh[4];
    const T r = reduce_parts(parts + (int64_t)blockIdx.x * np, np, sh);
    if (threadIdx.x == 0) out[blockIdx.x] = r;
}

// Single-launch reduction for short vectors (one 1024-thread block, fixed order).
template <typename T, int OP>
__global__ __launch_bounds__(1024) void k_reduce_single(int64_t n, const T* __restrict__ a,
                                                        const T* __restrict__ b, T* out) {
    __shared__ T sh[16];
    T acc = 0;
    for (int64_t i = threadIdx.x; i < n; i += 1024) {
        if (OP == 0) acc += a[i] * b[i];
        else if (OP == 1) acc += a[i] * a[i];
        else { T d = a[i] - b[i]; acc += d * d; }
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T r = 0;
        for (int w = 0; w < 16; ++w) r += sh[w];
        *out = r;
    }
}

constexpr int64_t SINGLE_MAX = 1 << 18;   // vectors up to 256 Ki entries: one launch

template <typename T, int OP>
static void reduce_to(hgm_ctx* c, int64_t n, const T* a, const T* b, T* out) {
    if (n <= SINGLE_MAX) {
        k_reduce_single<T, OP><<<1, 1024, 0, c->stream>>>(n, a, b, out);
        HGM_HIP(hipGetLastError());
        return;
    }
    const int np = parts_for(n);
    T* parts = c->buf<T>("red_parts", MAX_PARTS);
    k_reduce_partial<T, OP><<<np, BS, 0, c->stream>>>(n, a, b, parts);
    k_finalize<T><<<1, BS, 0, c->stream>>>(parts, np, out);
    HGM_HIP(hipGetLastError());
}

template <typename T> void dot(hgm_ctx* c, int64_t n, const T* a, const T* b, T* out) { reduce_to<T, 0>(c, n, a, b, out); }
template <typename T> void sumsq(hgm_ctx* c, int64_t n, const T* a, T* out) { reduce_to<T, 1>(c, n, a, a, out); }
template <typename T> void sumsq_diff(hgm_ctx* c, int64_t n, const T* a, const T* b, T* out) { reduce_to<T, 2>(c, n, a, b, out); }

// partial dots of every column j (blockIdx.y) with w; column index ncols (if launched)
// is the extra vector e
template <typename T>
__global__ __launch_bounds__(BS) void k_multidot(int64_t n, const T* __restrict__ Q, int64_t ldq,
                                                 const T* __restrict__ w, T* __restrict__ parts, int ncols,
                                                 const T* __restrict__ e) {
    __shared__ T sh[4];
    const T* q = (int)blockIdx.y < ncols ? Q + (int64_t)blockIdx.y * ldq : e;
    T acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
        acc += q[i] * w[i];
    T tot = block_sum_all(acc, sh);
    if (threadIdx.x == 0) parts[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = tot;
}

template <typename T>
void multidot(hgm_ctx* c, int64_t n, int ncols, const T* Q, int64_t ldq, const T* w, T* out, const T* extra) {
    const int nc = ncols + (extra ? 1 : 0);
    if (nc <= 0) return;
    const int np = parts_for(n);
    T* parts = c->buf<T>("mdot_parts", (size_t)np * nc);
    k_multidot<T><<<dim3(np, nc), BS, 0, c->stream>>>(n, Q, ldq, w, parts, ncols, extra);
    k_finalize<T><<<nc, BS, 0, c->stream>>>(parts, np, out);
    HGM_HIP(hipGetLastError());
}

// x = Q(:,0:k) y fused with the error monitor: parts[blk] = sum (x_i - xt_i)^2
template <typename T>
__global__ __launch_bounds__(BS) void k_gemv_err(int64_t n, int k, const T* __restrict__ Q, int64_t ldq,
                                                 const T* __restrict__ y, T* __restrict__ x,
                                                 const T* __restrict__ xt, T* __restrict__ parts) {
    __shared__ T sh[4];
    T acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
        T s = 0;
        for (int j = 0; j < k; ++j) s += Q[(int64_t)j * ldq + i] * y[j];
        x[i] = s;
        const T d = s - xt[i];
        acc += d * d;
    }
    const T tot = block_sum_all(acc, sh);
    if (threadIdx.x == 0) parts[blockIdx.x] = tot;
}

template <typename T>
void gemv_err(hgm_ctx* c, int64_t n, int k, const T* Q, int64_t ldq, const T* y, T* x, const T* xt, T* err_out) {
    const int np = parts_for(n);
    T* parts = c->buf<T>("gemv_parts", MAX_PARTS);
    k_gemv_err<T><<<np, BS, 0, c->stream>>>(n, k, Q, ldq, y, x, xt, parts);
    k_finalize<T><<<1, BS, 0, c->stream>>>(parts, np, err_out);
    HGM_HIP(hipGetLastError());
}

template <typename T>
__global__ __launch_bounds__(BS) void k_fro2(int64_t nnz, const T* __restrict__ v, double* parts) {
    __shared__ double sh[4];
    double acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * BS) {
        const double d = (double)v[i];
        acc += d * d;
    }
    double tot = block_sum_all(acc, sh);
    if (threadIdx.x == 0) parts[blockIdx.x] = tot;
}

template <typename T>
void fro2(hgm_ctx* c, const hgm_mat* M, double* out) {
    const int np = parts_for(M->nnz);
    double* parts = c->buf<double>("fro_parts", MAX_PARTS);
    k_fro2<T><<<np, BS, 0, c->stream>>>(M->nnz, reinterpret_cast<const T*>(M->val), parts);
    k_finalize<double><<<1, BS, 0, c->stream>>>(parts, np, out);
    HGM_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------
// Modified Gram-Schmidt, one fused pass per j (hybrid_*_rtp.m:20-24)
// MODE 0: acc = q_d . v                       (first inner product, :21 with j = 1)
// MODE 1: h = H(j-1); v -= h q_a; acc = q_d . v   (:22 for j-1 fused with :21 for j)
// MODE 2: h = H(k);   v -= h q_a; acc = v . v      (:22 for j = k fused with norm, :24)
// h comes from the previous pass's block partials (np_in > 0, single GPU) or from a
// device scalar already all-reduced across ranks (np_in == 0).
// ------------------------------------------------------------------------------
template <typename T, int MODE>
__global__ __launch_bounds__(BS) void k_mgs_pass(int64_t n, const T* __restrict__ qa,
                                                 const T* __restrict__ qd, T* __restrict__ v,
                                                 const T* __restrict__ pin, int np_in,
                                                 const T* hsrc, T* hdst, T* __restrict__ pout) {
    using T2 = typename V2<T>::t;
    __shared__ T sh[4];
    T h = 0;
    if (MODE != 0) {
        h = (np_in > 0) ? reduce_parts(pin, np_in, sh) : *hsrc;
        if (hdst != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *hdst = h;
    }
    T acc0 = 0, acc1 = 0;
    const int64_t n2 = n >> 1;
    const int64_t stride = (int64_t)gridDim.x * BS;
    T2* v2 = reinterpret_cast<T2*>(v);
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n2; i += stride) {
        T2 vv = v2[i];
        if (MODE != 0) {
            const T2 qq = reinterpret_cast<const T2*>(qa)[i];
            const T p0 = h * qq.x, p1 = h * qq.y;
            vv.x = vv.x - p0;
            vv.y = vv.y - p1;
            v2[i] = vv;
        }
        if (MODE == 2) {
            acc0 += vv.x * vv.x;
            acc1 += vv.y * vv.y;
        } else {
            const T2 dd = reinterpret_cast<const T2*>(qd)[i];
            acc0 += dd.x * vv.x;
            acc1 += dd.y * vv.y;
        }
    }
    if ((n & 1) && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        const int64_t i = n - 1;
        T vv = v[i];
        if (MODE != 0) {
            const T p0 = h * qa[i];
            vv = vv - p0;
            v[i] = vv;
        }
        acc0 += (MODE == 2) ? vv * vv : qd[i] * vv;
    }
    const T tot = block_sum_all(acc0 + acc1, sh);
    if (threadIdx.x == 0) pout[blockIdx.x] = tot;
}

// H(k+1,k) = sqrt(sum v^2);  if nonzero: q_{k+1} = v / H(k+1,k)   (hybrid_*_rtp.m:24-26)
template <typename T>
__global__ __launch_bounds__(BS) void k_mgs_normalize(int64_t n, T* __restrict__ v,
                                                      const T* __restrict__ pin, int np_in,
                                                      const T* ssrc, T* hdst) {
    using T2 = typename V2<T>::t;
    __shared__ T sh[4];
    const T ss = (np_in > 0) ? reduce_parts(pin, np_in, sh) : *ssrc;
    const T nrm = sqrt(ss);
    if (blockIdx.x == 0 && threadIdx.x == 0) *hdst = nrm;
    if (nrm == 0) return;
    const int64_t n2 = n >> 1;
    T2* v2 = reinterpret_cast<T2*>(v);
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n2; i += (int64_t)gridDim.x * BS) {
        T2 vv = v2[i];
        vv.x = vv.x / nrm;
        vv.y = vv.y / nrm;
        v2[i] = vv;
    }
    if ((n & 1) && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) v[n - 1] = v[n - 1] / nrm;
}

template <typename T>
void mgs(hgm_ctx* c, int64_t n, T* Q, int64_t ldq, int kk, T* Hcol, bool dist) {
    hipEvent_t t0 = nullptr;
    timing_begin(c, KC_MGS, &t0);
    const int np = parts_for(n);
    T* P = c->buf<T>("mgs_parts", 2 * MAX_PARTS);
    T* Pb[2] = {P, P + MAX_PARTS};
    T* v = Q + (int64_t)(kk + 1) * ldq;
    T* ss = c->buf<T>("mgs_ss", 4);
    hipStream_t st = c->stream;
    // pass 0: h_0 partials
    k_mgs_pass<T, 0><<<np, BS, 0, st>>>(n, nullptr, Q, v, nullptr, 0, nullptr, nullptr, Pb[0]);
    if (dist) {
        k_finalize<T><<<1, BS, 0, st>>>(Pb[0], np, Hcol + 0);
        allreduce(c, Hcol, 1);
    }
    for (int j = 1; j <= kk + 1; ++j) {
        const T* qa = Q + (int64_t)(j - 1) * ldq;
        T* pin = Pb[(j - 1) & 1];
        T* pout = Pb[j & 1];
        const int np_in = dist ? 0 : np;
        T* hdst = dist ? nullptr : Hcol + (j - 1);
        if (j <= kk) {
            const T* qd = Q + (int64_t)j * ldq;
            k_mgs_pass<T, 1><<<np, BS, 0, st>>>(n, qa, qd, v, pin, np_in, Hcol + (j - 1), hdst, pout);
            if (dist) {
                k_finalize<T><<<1, BS, 0, st>>>(pout, np, Hcol + j);
                allreduce(c, Hcol + j, 1);
            }
        } else {
            k_mgs_pass<T, 2><<<np, BS, 0, st>>>(n, qa, nullptr, v, pin, np_in, Hcol + (j - 1), hdst, pout);
            if (dist) {
                k_finalize<T><<<1, BS, 0, st>>>(pout, np, ss);
                allreduce(c, ss, 1);
            }
        }
    }
    {
        T* pin = Pb[(kk + 1) & 1];
        k_mgs_normalize<T><<<np, BS, 0, st>>>(n, v, pin, dist ? 0 : np, ss, Hcol + kk + 1);
    }
    HGM_HIP(hipGetLastError());
    // algorithmic bytes: (32k+24)n-style count for k+1 = kk+1 columns
    const double s = sizeof(T);
    const double bytes = s * n * (2.0 + 4.0 * kk + 3.0 + 2.0);
    timing_end(c, KC_MGS, t0, bytes);
}

// ------------------------------------------------------------------------------
// GEMV over the Krylov basis: x = Q(:,0:k) y  or  x -= Q y
// ------------------------------------------------------------------------------
template <typename T, int MODE>
__global__ __launch_bounds__(BS) void k_gemv(int64_t n, int k, const T* __restrict__ Q, int64_t ldq,
                                             const T* __restrict__ y, T* __restrict__ x) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
        T s = 0;
        for (int j = 0; j < k; ++j) s += Q[(int64_t)j * ldq + i] * y[j];
        if (MODE == 0) x[i] = s;
        else x[i] = x[i] - s;
    }
}

template <typename T>
void gemv(hgm_ctx* c, int64_t n, int k, const T* Q, int64_t ldq, const T* y, T* x, int mode) {
    int64_t nb = (n + BS - 1) / BS;
    if (nb > 8192) nb = 8192;
    if (nb < 1) nb = 1;
    if (mode == 0) k_gemv<T, 0><<<nb, BS, 0, c->stream>>>(n, k, Q, ldq, y, x);
    else k_gemv<T, 1><<<nb, BS, 0, c->stream>>>(n, k, Q, ldq, y, x);
    HGM_HIP(hipGetLastError());
}

// Classical Gram-Schmidt applied twice (option; C3's MGS vs CGS2 comparison).
template <typename T>
__global__ __launch_bounds__(BS) void k_add_store(int k, const T* a, const T* b, T* out) {
    const int i = threadIdx.x;
    if (i < k) out[i] = a[i] + b[i];
}

template <typename T>
void cgs2(hgm_ctx* c, int64_t n, T* Q, int64_t ldq, int kk, T* Hcol, bool dist) {
    hipEvent_t t0 = nullptr;
    timing_begin(c, KC_MGS, &t0);
    const int k = kk + 1;
    T* v = Q + (int64_t)k * ldq;
    T* h1 = c->buf<T>("cgs_h1", k + 8);
    T* h2 = c->buf<T>("cgs_h2", k + 8);
    multidot<T>(c, n, k, Q, ldq, v, h1, nullptr);
    if (dist) allreduce(c, h1, k);
    gemv<T>(c, n, k, Q, ldq, h1, v, 1);
    multidot<T>(c, n, k, Q, ldq, v, h2, nullptr);
    if (dist) allreduce(c, h2, k);
    gemv<T>(c, n, k, Q, ldq, h2, v, 1);
    k_add_store<T><<<1, BS, 0, c->stream>>>(k, h1, h2, Hcol);
    T* ss = c->buf<T>("mgs_ss", 4);
    sumsq<T>(c, n, v, ss);
    if (dist) allreduce(c, ss, 1);
    k_mgs_normalize<T><<<parts_for(n), BS, 0, c->stream>>>(n, v, nullptr, 0, ss, Hcol + k);
    HGM_HIP(hipGetLastError());
    const double s = sizeof(T);
    timing_end(c, KC_MGS, t0, s * n * (4.0 * k + 8.0));
}

// ------------------------------------------------------------------------------
// Elementwise
// ------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(BS) void k_div(int64_t n, const T* __restrict__ in, T* __restrict__ out, T s) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
        out[i] = in[i] / s;
}
template <typename T> void div_scalar(hgm_ctx* c, int64_t n, const T* in, T* out, T s) {
    k_div<T><<<grid_for(n), BS, 0, c->stream>>>(n, in, out, s);
    HGM_HIP(hipGetLastError());
}

// lsqr_solver.m:40-41:  x = x + (phi/rho) w ;  w = v - (theta/rho) w
template <typename T>
__global__ __launch_bounds__(BS) void k_lsqr_update(int64_t n, T* __restrict__ x, T* __restrict__ w,
                                                    const T* __restrict__ v, T a, T b) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
        const T wi = w[i];
        const T p = a * wi;
        x[i] = x[i] + p;
        const T q = b * wi;
        w[i] = v[i] - q;
    }
}
template <typename T> void lsqr_update(hgm_ctx* c, int64_t n, T* x, T* w, const T* v, T a, T b) {
    k_lsqr_update<T><<<grid_for(n), BS, 0, c->stream>>>(n, x, w, v, a, b);
    HGM_HIP(hipGetLastError());
}

// lsmr_solver.m:61-67
template <typename T, bool FIRST>
__global__ __launch_bounds__(BS) void k_lsmr_update(int64_t n, T* __restrict__ x, T* __restrict__ h,
                                                    T* __restrict__ hbar, const T* __restrict__ v,
                                                    T c_hbar, T c_x, T c_h) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
        const T hi = h[i];
        T hb;
        if (FIRST) hb = hi;                              // :62  hbar = h
        else { const T p = c_hbar * hbar[i]; hb = hi - p; }   // :64
        hbar[i] = hb;
        const T q = c_x * hb;
        x[i] = x[i] + q;                                 // :66
        const T r = c_h * hi;
        h[i] = v[i] - r;                                 // :67
    }
}
template <typename T>
void lsmr_update(hgm_ctx* c, int64_t n, T* x, T* h, T* hbar, const T* v, T c_hbar, T c_x, T c_h, bool first) {
    if (first) k_lsmr_update<T, true><<<grid_for(n), BS, 0, c->stream>>>(n, x, h, hbar, v, c_hbar, c_x, c_h);
    else k_lsmr_update<T, false><<<grid_for(n), BS, 0, c->stream>>>(n, x, h, hbar, v, c_hbar, c_x, c_h);
    HGM_HIP(hipGetLastError());
}

template <typename T>
__global__ __launch_bounds__(BS) void k_fill(int64_t n, T* x, T v) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) x[i] = v;
}
template <typename T> void fill(hgm_ctx* c, int64_t n, T* x, T v) {
    k_fill<T><<<grid_for(n), BS, 0, c->stream>>>(n, x, v);
    HGM_HIP(hipGetLastError());
}

template <typename T>
__global__ __launch_bounds__(BS) void k_convert(int64_t n, const double* in, T* out) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) out[i] = (T)in[i];
}
template <typename T>
__global__ __launch_bounds__(BS) void k_convert_back(int64_t n, const T* in, double* out) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) out[i] = (double)in[i];
}
template <typename T> void convert(hgm_ctx* c, int64_t n, const double* in, T* out) {
    k_convert<T><<<grid_for(n), BS, 0, c->stream>>>(n, in, out);
    HGM_HIP(hipGetLastError());
}
template <typename T> void convert_back(hgm_ctx* c, int64_t n, const T* in, double* out) {
    k_convert_back<T><<<grid_for(n), BS, 0, c->stream>>>(n, in, out);
    HGM_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------
// explicit instantiations
// ------------------------------------------------------------------------------
#define HGM_INST(T)                                                                            \
    template void dot<T>(hgm_ctx*, int64_t, const T*, const T*, T*);                           \
    template void sumsq<T>(hgm_ctx*, int64_t, const T*, T*);                                   \
    template void sumsq_diff<T>(hgm_ctx*, int64_t, const T*, const T*, T*);                    \
    template void multidot<T>(hgm_ctx*, int64_t, int, const T*, int64_t, const T*, T*, const T*); \
    template void gemv_err<T>(hgm_ctx*, int64_t, int, const T*, int64_t, const T*, T*, const T*, T*); \
    template void mgs<T>(hgm_ctx*, int64_t, T*, int64_t, int, T*, bool);                       \
    template void cgs2<T>(hgm_ctx*, int64_t, T*, int64_t, int, T*, bool);                      \
    template void gemv<T>(hgm_ctx*, int64_t, int, const T*, int64_t, const T*, T*, int);       \
    template void div_scalar<T>(hgm_ctx*, int64_t, const T*, T*, T);                           \
    template void lsqr_update<T>(hgm_ctx*, int64_t, T*, T*, const T*, T, T);                   \
    template void lsmr_update<T>(hgm_ctx*, int64_t, T*, T*, T*, const T*, T, T, T, bool);      \
    template void fill<T>(hgm_ctx*, int64_t, T*, T);                                           \
    template void convert<T>(hgm_ctx*, int64_t, const double*, T*);                            \
    template void convert_back<T>(hgm_ctx*, int64_t, const T*, double*);                       \
    template void fro2<T>(hgm_ctx*, const hgm_mat*, double*);

HGM_INST(double)
HGM_INST(float)

}  // namespace hgm
