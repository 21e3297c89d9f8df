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
#include <type_traits>

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
// Fixed-order sums (parity mode, HGM_OPT_PARITY; internal.h fixed_reduce).  The order is
// the one oracle/restatement.py's fixed_order() implements with numpy (cumsum is a
// sequential accumulation): 64-term chunks summed left to right, then 64-value chunks of
// those, then the remaining values left to right.  Each term is rounded on its own (no
// FMA: the library is built with -ffp-contract=off).  Throughput is not the point: one
// thread per chunk, strided loads.
// ------------------------------------------------------------------------------
constexpr int FIX_CH = 64;

template <typename T, int OP>
__device__ __forceinline__ T fixed_term(int64_t i, int64_t n1, const T* a1, const T* b1, const T* a2, const T* b2) {
    const T* a = i < n1 ? a1 : a2;
    const T* b = i < n1 ? b1 : b2;
    const int64_t j = i < n1 ? i : i - n1;
    if (OP == 0) return a[j] * b[j];
    if (OP == 1) return a[j] * a[j];
    const T d = a[j] - b[j];
    return d * d;
}

// level 1: c[t] = sequential sum of terms [64 t, 64 t + 64)
template <typename T, int OP>
__global__ __launch_bounds__(BS) void k_fixed_l1(int64_t n, int64_t n1, const T* a1, const T* b1, const T* a2,
                                                 const T* b2, T* c) {
    const int64_t t = (int64_t)blockIdx.x * BS + threadIdx.x;
    const int64_t i0 = t * FIX_CH;
    if (i0 >= n) return;
    const int64_t i1 = i0 + FIX_CH < n ? i0 + FIX_CH : n;
    T s = fixed_term<T, OP>(i0, n1, a1, b1, a2, b2);
    for (int64_t i = i0 + 1; i < i1; ++i) {
        const T p = fixed_term<T, OP>(i, n1, a1, b1, a2, b2);
        s = s + p;
    }
    c[t] = s;
}

// level 2 + final, one block: d[l] = sequential sum of c[64 l, 64 l + 64), then out = d_0 + d_1 + ...
template <typename T>
__global__ __launch_bounds__(BS) void k_fixed_l2(int64_t nc, const T* __restrict__ c, T* __restrict__ d, T* out) {
    const int64_t nd = (nc + FIX_CH - 1) / FIX_CH;
    for (int64_t l = threadIdx.x; l < nd; l += BS) {
        const int64_t j0 = l * FIX_CH, j1 = j0 + FIX_CH < nc ? j0 + FIX_CH : nc;
        T s = c[j0];
        for (int64_t j = j0 + 1; j < j1; ++j) s = s + c[j];
        d[l] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        T s = nd > 0 ? d[0] : T(0);
        for (int64_t l = 1; l < nd; ++l) s = s + d[l];
        st_sys(out, s);
    }
}

template <typename T, int OP>
static void fixed_reduce_op(hgm_ctx* c, int64_t n1, const T* a1, const T* b1, int64_t n2, const T* a2, const T* b2,
                            T* out) {
    const int64_t n = n1 + n2;
    const int64_t nc = (n + FIX_CH - 1) / FIX_CH;
    T* cbuf = c->buf<T>("fixed_c", nc + 1);
    T* dbuf = c->buf<T>("fixed_d", (nc + FIX_CH - 1) / FIX_CH + 1);
    if (nc > 0) {
        const int64_t g = (nc + BS - 1) / BS;
        k_fixed_l1<T, OP><<<(unsigned)g, BS, 0, c->stream>>>(n, n1, a1, b1, a2, b2, cbuf);
    }
    k_fixed_l2<T><<<1, BS, 0, c->stream>>>(nc, cbuf, dbuf, out);
    HGM_HIP(hipGetLastError());
}

template <typename T>
void fixed_reduce(hgm_ctx* c, int op, int64_t n1, const T* a1, const T* b1, int64_t n2, const T* a2, const T* b2,
                  T* out) {
    if (op == 0) fixed_reduce_op<T, 0>(c, n1, a1, b1, n2, a2, b2, out);
    else if (op == 1) fixed_reduce_op<T, 1>(c, n1, a1, a1, n2, a2, a2, out);
    else fixed_reduce_op<T, 2>(c, n1, a1, b1, n2, a2, b2, out);
}

// ------------------------------------------------------------------------------
// Reductions
// ------------------------------------------------------------------------------
// Grid-stride order of the elementwise kernels with a fused partial sum (VEC: 16-byte vectors of W
// elements -- thread g of the grid takes vectors g, g + G, ... and their elements in order, and the
// last block's thread 0 then the n mod W tail; else single elements g, g + G, ...).  Every kernel
// whose partials must give the same bits as another's (k_lsqr_step's error sum and
// k_reduce_partial<T, 2>) walks its elements through this.
template <typename T, bool VEC, typename F>
__device__ __forceinline__ void grid_elems(int64_t n, F&& f) {
    if constexpr (VEC) {
        using V = typename V16<T>::t;
        constexpr int W = V16<T>::W;
        (void)sizeof(V);
        const int64_t nv = n / W;
#pragma unroll 2
        for (int64_t g = (int64_t)blockIdx.x * BS + threadIdx.x; g < nv; g += (int64_t)gridDim.x * BS)
            f(g * W, std::integral_constant<int, W>{});
        if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
            for (int64_t i = nv * W; i < n; ++i) f(i, std::integral_constant<int, 1>{});
    } else {
        for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
            f(i, std::integral_constant<int, 1>{});
    }
}

// W consecutive elements from p + i (one 16-byte access for W > 1; i a multiple of W)
template <int W, typename T>
__device__ __forceinline__ void vload(const T* p, int64_t i, T (&o)[W]) {
    if constexpr (W == 1) {
        o[0] = p[i];
    } else {
        const typename V16<T>::t v = *reinterpret_cast<const typename V16<T>::t*>(p + i);
#pragma unroll
        for (int e = 0; e < W; ++e) o[e] = v[e];
    }
}
template <int W, typename T>
__device__ __forceinline__ void vstore(T* p, int64_t i, const T (&o)[W]) {
    if constexpr (W == 1) {
        p[i] = o[0];
    } else {
        typename V16<T>::t v;
#pragma unroll
        for (int e = 0; e < W; ++e) v[e] = o[e];
        *reinterpret_cast<typename V16<T>::t*>(p + i) = v;
    }
}

template <typename T, int OP, bool VEC>   // 0: a.b   1: a.a   2: (a-b).(a-b)
__global__ __launch_bounds__(BS) void k_reduce_partial(int64_t n, const T* __restrict__ a,
                                                       const T* __restrict__ b,
                                                       T* __restrict__ parts) {
    __shared__ T sh[4];
    T acc = 0;
    grid_elems<T, VEC>(n, [&](int64_t i, auto wc) {
        constexpr int W = decltype(wc)::value;
        T av[W], bv[W];
        vload<W>(a, i, av);
        if (OP != 1) vload<W>(b, i, bv);
#pragma unroll
        for (int e = 0; e < W; ++e) {
            if (OP == 0) acc += av[e] * bv[e];
            else if (OP == 1) acc += av[e] * av[e];
            else { T d = av[e] - bv[e]; acc += d * d; }
        }
    });
    T tot = block_sum_all(acc, sh);
    if (threadIdx.x == 0) parts[blockIdx.x] = tot;
}

template <typename T>
__global__ __launch_bounds__(BS) void k_finalize(const T* __restrict__ parts, int np, T* out) {
    __shared__ T sh[4];
    const T r = reduce_parts(parts + (int64_t)blockIdx.x * np, np, sh);
    if (threadIdx.x == 0) st_sys(out + blockIdx.x, r);
}

// Single-launch reduction for short vectors (one 1024-thread block, fixed order).
template <typename T, int OP>
__global__ __launch_bounds__(1024) void k_reduce_single(int64_t n, const T* __restrict__ a,
                                                        const T* __restrict__ b, T* out) {
    __shared__ T sh[16];
    // four independent loads in flight per lane (the loop is latency-bound, not HBM-bound)
    T a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    auto term = [&](int64_t i) -> T {
        if (OP == 0) return a[i] * b[i];
        if (OP == 1) return a[i] * a[i];
        const T d = a[i] - b[i];
        return d * d;
    };
    int64_t i = threadIdx.x;
    for (; i + 3 * 1024 < n; i += 4 * 1024) {
        const T t0 = term(i), t1 = term(i + 1024), t2 = term(i + 2048), t3 = term(i + 3072);
        a0 += t0;
        a1 += t1;
        a2 += t2;
        a3 += t3;
    }
    for (; i < n; i += 1024) a0 += term(i);
    T acc = (a0 + a1) + (a2 + a3);
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T r = 0;
        for (int w = 0; w < 16; ++w) r += sh[w];
        st_sys(out, r);
    }
}

constexpr int64_t SINGLE_MAX = 1 << 15;   // vectors up to 32 Ki entries: one launch

template <typename T, int OP>
static void reduce_to(hgm_ctx* c, int64_t n, const T* a, const T* b, T* out) {
    if (c->num.parity) {
        fixed_reduce_op<T, OP>(c, n, a, b, 0, nullptr, nullptr, out);
        return;
    }
    if (n <= SINGLE_MAX) {
        k_reduce_single<T, OP><<<1, 1024, 0, c->stream>>>(n, a, b, out);
        HGM_HIP(hipGetLastError());
        return;
    }
    const int np = parts_for(n);
    T* parts = c->buf<T>("red_parts", MAX_PARTS);
    if (al16(a) && al16(b)) k_reduce_partial<T, OP, true><<<np, BS, 0, c->stream>>>(n, a, b, parts);
    else k_reduce_partial<T, OP, false><<<np, BS, 0, c->stream>>>(n, a, b, parts);
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
    if (c->num.parity) {   // one fixed-order dot per column (the oracle's fixed_order() Q'w)
        for (int j = 0; j < ncols; ++j) fixed_reduce_op<T, 0>(c, n, Q + (int64_t)j * ldq, w, 0, nullptr, nullptr, out + j);
        if (extra) fixed_reduce_op<T, 0>(c, n, extra, w, 0, nullptr, nullptr, out + ncols);
        return;
    }
    const int np = parts_for(n);
    T* parts = c->buf<T>("mdot_parts", (size_t)np * nc);
    k_multidot<T><<<dim3(np, nc), BS, 0, c->stream>>>(n, Q, ldq, w, parts, ncols, extra);
    k_finalize<T><<<nc, BS, 0, c->stream>>>(parts, np, out);
    HGM_HIP(hipGetLastError());
}

// ------------------------------------------------------------------------------
// GEMV over the Krylov basis, x = Q(:,0:k) y (MODE 0), x -= Q y (MODE 1), or MODE 0
// fused with the error monitor (ERR: parts[blk] = sum (x_i - xt_i)^2).  y (k values,
// possibly in pinned host memory written by the projected solve) is staged once per
// block in LDS; every lane owns a pair of rows and keeps four column loads in flight.
// The sum over j runs in increasing j (s = ((q0 y0 + q1 y1) + q2 y2) + ...).
// ------------------------------------------------------------------------------
constexpr int GEMV_KMAX = 8192;   // LDS staging of y (64 KiB of doubles)

// Rows [blk*BS .. ) of a block-range [0, nblk) of the GEMV s = Q(:,0:k) y with y staged in
// LDS (ys).  MODE 0: x = s ; MODE 1: x = x - s ; MODE 2: nothing written.  ACC: returns
// this lane's sum of (s_i - z_i)^2 (the error monitor with z = x_true, or the residual
// monitor norm(b - A*x)^2 with Q = A*Q, z = b).
template <typename T, int MODE, bool ACC>
__device__ __forceinline__ T gemv_rows(int64_t n, int k, const T* __restrict__ Q, int64_t ldq, const T* ys,
                                       T* __restrict__ x, const T* __restrict__ z, int64_t blk, int64_t nblk) {
    using T2 = typename V2<T>::t;
    T acc = 0;
    const int64_t n2 = n >> 1;
    const int64_t stride = nblk * BS;
    const int64_t ld2 = ldq >> 1;
    for (int64_t i = blk * BS + threadIdx.x; i < n2; i += stride) {
        const T2* q2 = reinterpret_cast<const T2*>(Q) + i;
        T s0 = 0, s1 = 0;
        int j = 0;
        for (; j + 4 <= k; j += 4) {
            const T2 a = q2[(int64_t)j * ld2], b = q2[(int64_t)(j + 1) * ld2];
            const T2 cc = q2[(int64_t)(j + 2) * ld2], d = q2[(int64_t)(j + 3) * ld2];
            s0 += a.x * ys[j];
            s1 += a.y * ys[j];
            s0 += b.x * ys[j + 1];
            s1 += b.y * ys[j + 1];
            s0 += cc.x * ys[j + 2];
            s1 += cc.y * ys[j + 2];
            s0 += d.x * ys[j + 3];
            s1 += d.y * ys[j + 3];
        }
        for (; j < k; ++j) {
            const T2 a = q2[(int64_t)j * ld2];
            s0 += a.x * ys[j];
            s1 += a.y * ys[j];
        }
        if (MODE == 0) {
            reinterpret_cast<T2*>(x)[i] = T2{s0, s1};
        } else if (MODE == 1) {
            T2 xv = reinterpret_cast<T2*>(x)[i];
            xv.x = xv.x - s0;
            xv.y = xv.y - s1;
            reinterpret_cast<T2*>(x)[i] = xv;
        }
        if (ACC) {
            const T2 t = reinterpret_cast<const T2*>(z)[i];
            const T d0 = s0 - t.x, d1 = s1 - t.y;
            acc += d0 * d0;
            acc += d1 * d1;
        }
    }
    if ((n & 1) && blk == nblk - 1 && threadIdx.x == 0) {
        const int64_t i = n - 1;
        T s = 0;
        for (int j = 0; j < k; ++j) s += Q[(int64_t)j * ldq + i] * ys[j];
        if (MODE == 0) x[i] = s;
        else if (MODE == 1) x[i] = x[i] - s;
        if (ACC) { const T d = s - z[i]; acc += d * d; }
    }
    return acc;
}

template <typename T>
__device__ __forceinline__ T* stage_y(const T* __restrict__ y, int k) {
    extern __shared__ unsigned char gemv_smem[];
    T* ys = reinterpret_cast<T*>(gemv_smem);
    for (int j = threadIdx.x; j < k; j += BS) ys[j] = y[j];
    __syncthreads();
    return ys;
}

template <typename T, int MODE, bool ERR>
__global__ __launch_bounds__(BS) void k_gemv2(int64_t n, int k, const T* __restrict__ Q, int64_t ldq,
                                              const T* __restrict__ y, T* __restrict__ x,
                                              const T* __restrict__ xt, T* __restrict__ parts) {
    __shared__ T sh[4];
    const T* ys = stage_y(y, k);
    const T acc = gemv_rows<T, MODE, ERR>(n, k, Q, ldq, ys, x, xt, blockIdx.x, gridDim.x);
    if (ERR) {
        const T tot = block_sum_all(acc, sh);
        if (threadIdx.x == 0) parts[blockIdx.x] = tot;
    }
}

// GMRES reconstruction of iteration k in one launch (n-space side): blocks [0, nbx)
// compute x = Q(:,0:k) y with the error monitor sum (x - x_true)^2; blocks [nbx, grid)
// the residual monitor sum (b - AQ(:,0:k) y)^2 over the m rows (A*x = (A*Q) y: the
// columns A*Q(:,j) are the operator's own products, kept from the Arnoldi steps).
template <typename T>
__global__ __launch_bounds__(BS) void k_recon(int64_t n, int k, const T* __restrict__ Q, int64_t ldq,
                                              const T* __restrict__ y, T* __restrict__ x, const T* __restrict__ xt,
                                              int64_t m, const T* __restrict__ AQ, int64_t ldaq,
                                              const T* __restrict__ b, T* __restrict__ parts, int nbx) {
    __shared__ T sh[4];
    const T* ys = stage_y(y, k);
    T acc;
    if ((int)blockIdx.x < nbx) acc = gemv_rows<T, 0, true>(n, k, Q, ldq, ys, x, xt, blockIdx.x, nbx);
    else acc = gemv_rows<T, 2, true>(m, k, AQ, ldaq, ys, nullptr, b, blockIdx.x - nbx, gridDim.x - nbx);
    const T tot = block_sum_all(acc, sh);
    if (threadIdx.x == 0) parts[blockIdx.x] = tot;
}

// block 0: out0 = sum parts[0, n0) ; block 1: out1 = sum parts[n0, n0 + n1)
template <typename T>
__global__ __launch_bounds__(BS) void k_finalize2(const T* __restrict__ parts, int n0, int n1, T* out0, T* out1) {
    __shared__ T sh[4];
    const T r = blockIdx.x == 0 ? reduce_parts(parts, n0, sh) : reduce_parts(parts + n0, n1, sh);
    if (threadIdx.x == 0) st_sys(blockIdx.x == 0 ? out0 : out1, r);
}

static int gemv_blocks(int64_t n, int ppl = 1) {
    const int64_t per = (int64_t)BS * ppl;
    int64_t nb = ((n >> 1) + per - 1) / per;  // ppl row pairs per lane ...
    if (nb > MAX_PARTS) nb = MAX_PARTS;      // ... up to 1024 blocks, then grid-stride
    if (nb < 1) nb = 1;
    return (int)nb;
}

// row pairs per lane of the MGS passes (HGM_OPT_MGS_PPL; default 1)
static int mgs_ppl(const hgm_ctx* c) { return c->num.mgs_ppl > 0 ? c->num.mgs_ppl : 1; }

template <typename T>
void gemv_err(hgm_ctx* c, int64_t n, int k, const T* Q, int64_t ldq, const T* y, T* x, const T* xt, T* err_out) {
    HGM_REQUIRE(k <= GEMV_KMAX && ldq % 2 == 0, "gemv: k too large");
    if (c->num.parity) {   // x = Q y (sequential over the columns), then the fixed-order error norm
        gemv<T>(c, n, k, Q, ldq, y, x, 0);
        fixed_reduce_op<T, 2>(c, n, x, xt, 0, nullptr, nullptr, err_out);
        return;
    }
    const int np = gemv_blocks(n);
    T* parts = c->buf<T>("gemv_parts", MAX_PARTS);
    k_gemv2<T, 0, true><<<np, BS, sizeof(T) * (k > 0 ? k : 1), c->stream>>>(n, k, Q, ldq, y, x, xt, parts);
    k_finalize<T><<<1, BS, 0, c->stream>>>(parts, np, err_out);
    HGM_HIP(hipGetLastError());
}

template <typename T>
void recon(hgm_ctx* c, int64_t n, int k, const T* Q, int64_t ldq, const T* y, T* x, const T* xt, T* err_out,
           int64_t m, const T* AQ, int64_t ldaq, const T* b, T* res_out) {
    HGM_REQUIRE(k <= GEMV_KMAX && ldq % 2 == 0 && ldaq % 2 == 0, "recon: k too large");
    HGM_REQUIRE(!c->num.parity, "recon: parity mode forms the monitors explicitly");
    // x == nullptr: the residual monitor only (the error comes from the Gram error monitor)
    const int nbx = x ? gemv_blocks(n) : 0, nbr = gemv_blocks(m);
    T* parts = c->buf<T>("recon_parts", 2 * MAX_PARTS);
    if (!x) err_out = c->buf<T>("recon_noerr", 2);
    k_recon<T><<<nbx + nbr, BS, sizeof(T) * (k > 0 ? k : 1), c->stream>>>(n, k, Q, ldq, y, x, xt, m, AQ, ldaq, b,
                                                                          parts, nbx);
    k_finalize2<T><<<2, BS, 0, c->stream>>>(parts, nbx, nbr, err_out, res_out);
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
__global__ __launch_bounds__(BS) void k_to_f64(int64_t n, const T* __restrict__ in, double* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) out[i] = (double)in[i];
}

template <typename T>
void fro2(hgm_ctx* c, const hgm_mat* M, double* out) {
    if (c->num.parity) {   // norm(A,'fro')^2 over the stored values, in double, fixed order
        const double* v = reinterpret_cast<const double*>(M->val);
        if (!std::is_same<T, double>::value) {                 // fp32 values, widened exactly
            double* w = c->buf<double>("fro_f64", M->nnz + 1);
            k_to_f64<T><<<grid_for(M->nnz), BS, 0, c->stream>>>(M->nnz, reinterpret_cast<const T*>(M->val), w);
            v = w;
        }
        fixed_reduce_op<double, 1>(c, M->nnz, v, v, 0, nullptr, nullptr, out);
        return;
    }
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
// Side job of an MGS pass (MdotJob): stage 1 = the multidot partials of block g (the
// k_multidot block (g % np, g / np)), stage 2 = the finalize of column g (k_finalize).
template <typename T>
struct MdotStage {
    MdotJob<T> j;
    int np = 0;          // partial blocks per column
    T* parts = nullptr;
    int stage = 0;       // 0: none
    int blocks() const { return stage == 1 ? np * (j.ncols + 1) : stage == 2 ? j.ncols + 1 : 0; }
};

template <typename T>
__device__ __forceinline__ void mdot_side(const MdotStage<T>& S, int g, T* sh) {
    if (S.stage == 1) {
        const int col = g / S.np, p = g - col * S.np;
        const T* q = col < S.j.ncols ? S.j.Q + (int64_t)col * S.j.ldq : S.j.e;
        T acc = 0;
        for (int64_t i = (int64_t)p * BS + threadIdx.x; i < S.j.n; i += (int64_t)S.np * BS) acc += q[i] * S.j.w[i];
        const T tot = block_sum_all(acc, sh);
        if (threadIdx.x == 0) S.parts[(int64_t)col * S.np + p] = tot;
    } else {
        const T r = reduce_parts(S.parts + (int64_t)g * S.np, S.np, sh);
        if (threadIdx.x == 0) st_sys(S.j.out + g, r);
    }
}

template <typename T, int MODE>
__global__ __launch_bounds__(BS) void k_mgs_pass(int64_t n, int nb, const T* __restrict__ qa,
                                                 const T* __restrict__ qd, const T* vin, T* v,
                                                 const T* __restrict__ pin, int np_in,
                                                 const T* hsrc, T* hdst, T* __restrict__ pout,
                                                 MdotStage<T> side) {
    using T2 = typename V2<T>::t;
    __shared__ T sh[4], sh2[4];   // one LDS slot set per reduction: no trailing barriers
    if ((int)blockIdx.x >= nb) {   // extra workgroups: the side job
        mdot_side(side, (int)blockIdx.x - nb, sh);
        return;
    }
    const int64_t n2 = n >> 1;
    const int64_t stride = (int64_t)nb * BS;
    const T2* vi2 = reinterpret_cast<const T2*>(vin);   // the vector before this pass (v or src)
    T2* v2 = reinterpret_cast<T2*>(v);
    const T2* qa2 = reinterpret_cast<const T2*>(qa);
    const T2* qd2 = reinterpret_cast<const T2*>(qd);
    // The first pair's loads do not depend on h: issue them before the re-reduction of
    // the previous pass's partials so the two latencies overlap.
    int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x;
    T2 vv{0, 0}, qq{0, 0}, dd{0, 0};
    if (i < n2) {
        vv = vi2[i];
        if (MODE != 0) qq = qa2[i];
        if (MODE != 2) dd = qd2[i];
    }
    T h = 0;
    if (MODE != 0) {
        h = (np_in > 0) ? reduce_parts<T, false>(pin, np_in, sh) : *hsrc;
        if (hdst != nullptr && blockIdx.x == 0 && threadIdx.x == 0) st_sys(hdst, h);
    }
    T acc0 = 0, acc1 = 0;
    while (i < n2) {
        if (MODE != 0) {
            const T p0 = h * qq.x, p1 = h * qq.y;
            vv.x = vv.x - p0;
            vv.y = vv.y - p1;
            v2[i] = vv;
        }
        if (MODE == 2) {
            acc0 += vv.x * vv.x;
            acc1 += vv.y * vv.y;
        } else {
            acc0 += dd.x * vv.x;
            acc1 += dd.y * vv.y;
        }
        i += stride;
        if (i < n2) {
            vv = vi2[i];
            if (MODE != 0) qq = qa2[i];
            if (MODE != 2) dd = qd2[i];
        }
    }
    if ((n & 1) && (int)blockIdx.x == nb - 1 && threadIdx.x == 0) {
        const int64_t i = n - 1;
        T vv = vin[i];
        if (MODE != 0) {
            const T p0 = h * qa[i];
            vv = vv - p0;
            v[i] = vv;
        }
        acc0 += (MODE == 2) ? vv * vv : qd[i] * vv;
    }
    const T tot = block_sum_all<T, false>(acc0 + acc1, sh2);
    if (threadIdx.x == 0) pout[blockIdx.x] = tot;
}

// H(k+1,k) = sqrt(sum v^2);  if nonzero: q_{k+1} = v / H(k+1,k)   (hybrid_*_rtp.m:24-26)
template <typename T>
__global__ __launch_bounds__(BS) void k_mgs_normalize(int64_t n, T* __restrict__ v,
                                                      const T* __restrict__ pin, int np_in,
                                                      const T* ssrc, T* hdst) {
    using T2 = typename V2<T>::t;
    __shared__ T sh[4];
    const int64_t n2 = n >> 1;
    T2* v2 = reinterpret_cast<T2*>(v);
    int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x;
    T2 vv{0, 0};
    if (i < n2) vv = v2[i];                       // overlaps the partial re-reduction
    const T ss = (np_in > 0) ? reduce_parts<T, false>(pin, np_in, sh) : *ssrc;
    const T nrm = sqrt(ss);
    if (blockIdx.x == 0 && threadIdx.x == 0) st_sys(hdst, nrm);
    if (nrm == 0) return;
    while (i < n2) {
        vv.x = vv.x / nrm;
        vv.y = vv.y / nrm;
        v2[i] = vv;
        i += (int64_t)gridDim.x * BS;
        if (i < n2) vv = v2[i];
    }
    if ((n & 1) && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) v[n - 1] = v[n - 1] / nrm;
}

// Whole MGS sweep of a short vector in ONE workgroup (hybrid_*_rtp.m:20-26): v lives in
// registers (E entries per lane, entry t + 1024 j), each pass reads q_i once, and the
// inner product is a wave butterfly + 16-wave LDS sum read back by every lane in the
// same order, so every lane holds identical h_i.  Replaces kk+3 dependent launches
// (~4.9 us each at m = 21750) with one; the other CUs stay free for the aux stream.
// The basis is stored with ldq = 1024 E and zero padding past n (krylov_ld), so the
// kernel reads and writes whole 1024-entry chunks of the basis with no bounds checks (padding stays
// zero: 0 - h 0 = 0, 0 / nrm = 0).  The LDS slots alternate between passes so one
// barrier per pass suffices.
constexpr int MGS1_BS = 1024;
constexpr int64_t MGS1_MAX = 24 * MGS1_BS;   // E <= 24: w and q fit 4E = 96 VGPRs
template <typename T, int E>
__global__ __launch_bounds__(MGS1_BS) void k_mgs_single(int n, const T* __restrict__ Q, int64_t ldq, const T* src,
                                                        T* v, int kk, T* __restrict__ Hcol) {
    __shared__ T sh[2][MGS1_BS / 64];
    const int t = threadIdx.x;
    // one buffer resource per column; chunk j is the constant soffset j * 1024 * sizeof(T),
    // so every load and store shares the single lane-offset VGPR
    const int off = t * (int)sizeof(T);
    constexpr int CH = MGS1_BS * (int)sizeof(T);
    const int bytes = (int)ldq * (int)sizeof(T);
    auto ldc = [&](__amdgpu_buffer_rsrc_t r, int j) -> T {
        if constexpr (sizeof(T) == 8)
            return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, off, j * CH, 0));
        else
            return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, off, j * CH, 0));
    };
    T w[E], q[E];
    const __amdgpu_buffer_rsrc_t rv = buf_rsrc(v, bytes);
    // src may be another array's column (no zero padding past n): bounds-checked loads
#pragma unroll
    for (int j = 0; j < E; ++j) {
        const int i = t + MGS1_BS * j;
        w[j] = i < n ? src[i] : T(0);
    }
    // block sum: DPP wave sum, one LDS slot per wave, then a DPP sum of the 16 slots in
    // every row (every lane, hence every wave, gets the same bits)
    auto bsum = [&](T a, int slot) -> T {
        static_assert(MGS1_BS / 64 == 16, "one LDS slot per wave, one 16-lane row");
        a = wave_sum_dpp(a);
        if ((t & 63) == 0) sh[slot][t >> 6] = a;
        __syncthreads();
        return row16_sum(sh[slot][t & 15]);
    };
    // kk >= 0: a do-while keeps w in one register set (a zero-trip-capable loop makes
    // the compiler copy the loaded w and spill at E = 24)
    int p = 0;
    do {
        const __amdgpu_buffer_rsrc_t rq = buf_rsrc(Q + (int64_t)p * ldq, bytes);
#pragma unroll
        for (int j = 0; j < E; ++j) q[j] = ldc(rq, j);
        // fused multiply-adds keep the partial dot in two registers (the products are
        // not held while the loads drain)
        T a0 = 0, a1 = 0;
#pragma unroll
        for (int j = 0; j < E; j += 2) {
            a0 = __builtin_fma(q[j], w[j], a0);
            a1 = __builtin_fma(q[j + 1], w[j + 1], a1);
        }
        const T h = bsum(a0 + a1, p & 1);
        if (t == 0) st_sys(Hcol + p, h);
#pragma unroll
        for (int j = 0; j < E; ++j) {
            const T s = h * q[j];
            w[j] = w[j] - s;
        }
    } while (++p <= kk);
    T a0 = 0, a1 = 0;
#pragma unroll
    for (int j = 0; j < E; j += 2) {
        a0 = __builtin_fma(w[j], w[j], a0);
        a1 = __builtin_fma(w[j + 1], w[j + 1], a1);
    }
    const T nrm = sqrt(bsum(a0 + a1, (kk + 1) & 1));
    if (t == 0) st_sys(Hcol + kk + 1, nrm);
    if (nrm != 0) {
#pragma unroll
        for (int j = 0; j < E; ++j) w[j] = w[j] / nrm;
    }
#pragma unroll
    for (int j = 0; j < E; ++j) {
        if constexpr (sizeof(T) == 8)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(rv, 0, 0, 0)), w[j]), rv, off, j * CH, 0);
        else
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b32(rv, 0, 0, 0)), w[j]), rv, off, j * CH, 0);
    }
}

// one-workgroup sweep for short bases (HGM_OPT_MGS_SINGLE; never in parity mode)
static bool mgs_single_on(const hgm_ctx* c) { return c->num.mgs_single && !c->num.parity; }

int64_t krylov_ld(const hgm_ctx* c, int64_t dim, bool dist) {
    dim = dim > 0 ? dim : 1;
    if (!dist && dim <= MGS1_MAX && mgs_single_on(c)) return (dim + 4 * MGS1_BS - 1) / (4 * MGS1_BS) * (4 * MGS1_BS);
    const int64_t ld = (dim + 63) / 64 * 64;
    // a column stride that is a multiple of 32 KiB (C3: 2048^2 pixels, 32 MiB) puts element i of
    // every column in the same HBM channel: the sweeps read k+2 columns at the same i at once
    const int pad = c->num.krylov_pad < 0 ? 0 : c->num.krylov_pad;   // (auto: none)
    return ld % 4096 == 0 ? ld + pad : ld;
}

bool krylov_padded(const hgm_ctx* c, int64_t ldq) {
    return ldq % (4 * MGS1_BS) == 0 && ldq <= MGS1_MAX && mgs_single_on(c);
}

template <typename T>
static bool mgs_single(hgm_ctx* c, int64_t n, T* Q, int64_t ldq, int kk, T* Hcol, const T* src) {
    if (!krylov_padded(c, ldq) || n > ldq) return false;
    T* v = Q + (int64_t)(kk + 1) * ldq;
    hipStream_t st = c->stream;
    switch (ldq / MGS1_BS) {
    case 4: k_mgs_single<T, 4><<<1, MGS1_BS, 0, st>>>((int)n, Q, ldq, src, v, kk, Hcol); break;
    case 8: k_mgs_single<T, 8><<<1, MGS1_BS, 0, st>>>((int)n, Q, ldq, src, v, kk, Hcol); break;
    case 12: k_mgs_single<T, 12><<<1, MGS1_BS, 0, st>>>((int)n, Q, ldq, src, v, kk, Hcol); break;
    case 16: k_mgs_single<T, 16><<<1, MGS1_BS, 0, st>>>((int)n, Q, ldq, src, v, kk, Hcol); break;
    case 20: k_mgs_single<T, 20><<<1, MGS1_BS, 0, st>>>((int)n, Q, ldq, src, v, kk, Hcol); break;
    case 24: k_mgs_single<T, 24><<<1, MGS1_BS, 0, st>>>((int)n, Q, ldq, src, v, kk, Hcol); break;
    default: return false;
    }
    HGM_HIP(hipGetLastError());
    return true;
}

// ------------------------------------------------------------------------------
// MGS in one-reduction form (hybrid_*_rtp.m:20-26) for long vectors.  In exact
// arithmetic the MGS coefficients satisfy h_j = q_j'w - sum_{i<j} h_i (q_j'q_i) for ANY
// basis, orthonormal or not: (I + L) h = Q'w with L the strictly lower part of Q'Q (the
// "inverse compact WY" form of MGS, Swirydowicz, Langou, Ananthan, Yang, Thomas, Numer.
// Linear Algebra Appl. 28 (2021) e2343).  The sweep becomes four launches instead of k+3:
//   1. k_mgs1_dots   : block partials of Q(:,0:k)'w and of the new Gram row q_k'Q(:,0:k-1)
//   2. k_mgs1_solve  : one 1024-thread workgroup sums the 2k+1 partial rows (16 lanes per
//                      row, all loads in flight at once) and runs the forward substitution
//                      for h (Gram triangle in LDS)
//   3. k_mgs1_update : v = ((w - h_0 q_0) - h_1 q_1) - ... (MGS's own per-element order and
//                      roundings) with the norm partials
//   4. k_mgs_normalize (shared with the pass form)
// Summing the partials inside the dots kernel instead (last-arriving block per column
// group, device-scope fences) measured 2.4x slower at C2: every fence writes back and
// invalidates the XCD's L2.
// The basis is read twice instead of in 2(k+1) vector passes.  Only the dot products round
// differently from sequential MGS: |dH|/|H| = 8e-13 at k = 20 and 1.2e-11 at k = 80 on the
// tomography operators, the size of MGS's own sensitivity to the order of its dot-product
// sums.  Every sum has a fixed order, so results are bitwise reproducible.
// Multi-GPU: the 2k+1 sums are one all-reduce (the pass form needs k+1 all-reduces per
// step) between the two halves of k_mgs1_solve.
// ------------------------------------------------------------------------------
constexpr int MGS1_MAXC = 120;   // k+1 <= 120: the Gram triangle fits 57 KiB of LDS

// HGM_OPT_MGS_FORM: 1 = one-reduction (default), 0 = one launch per pass
static int mgs1_mode(const hgm_ctx* c) { return c->num.mgs_form; }
bool mgs_gram_ok(const hgm_ctx* c, int64_t ldq, int maxit, bool dist) {
    return !dist && !c->num.parity && maxit <= MGS1_MAXC && mgs1_mode(c) == 1 && !krylov_padded(c, ldq);
}
// Element pairs per lane of the sweep's tiles (HGM_OPT_MGS1_PPL; 0: by length).  A workgroup sweeps
// one tile of BS * P pairs at a time, and the grid has one workgroup per tile (up to MAX_PARTS, then
// grid-stride).  4 pairs per lane from n = 2^20 on (>= 512 tiles); shorter vectors take 2 (C2,
// n = 2^18: the sweep 19.2 us per step against 20.6 with 4 and 21.7 with 1, whose 512 partial rows
// every update workgroup sums again; profiles/r4_c2_mgs_tile_ab.jsonl).
static int mgs1_tile(const hgm_ctx* c, int64_t n) {
    if (c->num.mgs1_ppl > 0) return c->num.mgs1_ppl;
    const int64_t n2 = n >> 1;
    return n2 >= (int64_t)BS * 4 * 512 ? 4 : n2 >= (int64_t)BS * 2 * 128 ? 2 : 1;
}
static int mgs1_blocks(int64_t n, int P) {
    const int64_t tp = (int64_t)BS * P, nt = ((n >> 1) + tp - 1) / tp;
    return (int)std::max<int64_t>(1, std::min<int64_t>(nt, MAX_PARTS));
}

// Forward substitution (I + L) h = r in wave 0 (rows j = lane, lane + 64):
// s_j = ((r_j - h_0 G_j0) - h_1 G_j1) - ...;  h_i = s_i once rows < i are applied.
// sr: r (LDS), sG: packed strictly lower Gram triangle (LDS, row j at j(j-1)/2).
// h goes to device memory only: the update kernel's block 0 copies it to the host ring
// (a one-block kernel would wait at its end for the host-memory stores to complete).
template <typename T>
__device__ __forceinline__ void mgs1_substitute(int kk, const T* sr, const T* sG, T* hdev) {
    const int lane = threadIdx.x & 63;
    const int j0 = lane, j1 = lane + 64;
    T s0 = j0 <= kk ? sr[j0] : T(0);
    T s1 = j1 <= kk ? sr[j1] : T(0);
    const int o0 = j0 * (j0 - 1) / 2, o1 = j1 * (j1 - 1) / 2;
    // four steps per round: the Gram loads of a round are issued before its dependent chain
    for (int i0 = 0; i0 <= kk; i0 += 4) {
        T g0[4], g1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + u;
            g0[u] = (j0 > i && j0 <= kk) ? sG[o0 + i] : T(0);
            g1[u] = (j1 > i && j1 <= kk) ? sG[o1 + i] : T(0);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + u;
            if (i > kk) break;
            const T h = i < 64 ? lane_bcast(s0, i) : lane_bcast(s1, i - 64);
            if (lane == 0) hdev[i] = h;
            if (j0 > i && j0 <= kk) {
                const T p = h * g0[u];
                s0 = s0 - p;
            }
            if (j1 > i && j1 <= kk) {
                const T p = h * g1[u];
                s1 = s1 - p;
            }
        }
    }
}

// hpend (pending normalisation, internal.h PendNorm): Q(:,k) still holds v_k; every block
// uses q_k = v_k / *hpend (k_mgs1_update writes q_k back once this kernel is done).
// Tiles of BS*P element pairs per block (block b: tiles b, b + npr, ...).  A tile's w and q_k
// stay in registers while its columns stream past two at a time, so w and q_k are read once per
// step (the column-group form read them once per 8 columns) and a block streams two columns at a
// time.  Per column the tile's partial dot products are wave-summed (DPP, fixed order) and added
// into the block's LDS accumulators in tile order: fixed order, bitwise reproducible.
template <typename T, int P>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(4))) void k_mgs1_dots(
    int64_t n, const T* Q, int64_t ldq, int kk, const T* __restrict__ w, int npr, T* __restrict__ pr,
    T* __restrict__ pg, MdotStage<T> side, const T* hpend, const T* __restrict__ xe, const double* cp_src,
    double* cp_dst) {
    using T2 = typename V2<T>::t;
    constexpr int NW = BS / 64;
    if (cp_dst && blockIdx.x == 0 && threadIdx.x == 0) st_sys(cp_dst, *cp_src);   // (mgs: the ring copy)
    // acc[row][wave]: rows 0..kk = q_c'w, kk+1.. = q_c'q_k (c < kk; with xe also c = kk, then
    // q_k'x_true)
    __shared__ T acc[2 * MGS1_MAXC + 2][NW];
    const int b = (int)blockIdx.x;
    if (b >= npr) {   // extra workgroups: the side job
        mdot_side(side, b - npr, &acc[0][0]);
        return;
    }
    const bool gx = xe != nullptr;
    const int nrow = 2 * kk + 1 + (gx ? 2 : 0);
    const int t = threadIdx.x, wv = t >> 6, lane = t & 63;
    for (int r = t; r < nrow * NW; r += BS) (&acc[0][0])[(r / NW) * NW + r % NW] = T(0);
    __syncthreads();
    const T hp = hpend ? *hpend : T(0);
    auto scale = [&](T v) -> T { return hp != T(0) ? v / hp : v; };   // as k_mgs_normalize
    const int64_t n2 = n >> 1, tp = (int64_t)BS * P, ntile = (n2 + tp - 1) / tp, ld2 = ldq >> 1;
    auto add = [&](int row, T v) {              // one wave's share of a tile's partial
        const T sv = wave_sum_dpp(v);
        if (lane == 0) acc[row][wv] += sv;
    };
    for (int64_t tl = b; tl < ntile; tl += npr) {
        const int lim = (int)min<int64_t>(tp, n2 - tl * tp);
        int ix[P];
        bool ok[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const int e = t + p * BS;
            ok[p] = e < lim;
            ix[p] = ok[p] ? e : lim - 1;
        }
        const T2* wt = reinterpret_cast<const T2*>(w) + tl * tp;
        const T2* qt = reinterpret_cast<const T2*>(Q) + tl * tp;
        T2 ww[P], qk[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            ww[p] = ok[p] ? wt[ix[p]] : T2{0, 0};
            qk[p] = qt[(int64_t)kk * ld2 + ix[p]];
            if (hpend) {
                qk[p].x = scale(qk[p].x);
                qk[p].y = scale(qk[p].y);
            }
            if (!ok[p]) qk[p] = T2{0, 0};
        }
        auto col = [&](const T2 (&q)[P], int c) {
            T a = 0, g = 0;
#pragma unroll
            for (int p = 0; p < P; ++p) {
                a = __builtin_fma(q[p].y, ww[p].y, __builtin_fma(q[p].x, ww[p].x, a));
                g = __builtin_fma(q[p].y, qk[p].y, __builtin_fma(q[p].x, qk[p].x, g));
            }
            add(c, a);
            if (c < kk || gx) add(kk + 1 + c, g);
        };
        auto load = [&](int c, T2 (&q)[P]) {
            if (hpend && c == kk) {
#pragma unroll
                for (int p = 0; p < P; ++p) q[p] = qk[p];
                return;
            }
            const __amdgpu_buffer_rsrc_t rc = buf_rsrc(qt + (int64_t)c * ld2, lim * (int)sizeof(T2));
#pragma unroll
            for (int p = 0; p < P; ++p) q[p] = buf_load2<T2>(rc, (ok[p] ? ix[p] : lim) * (int)sizeof(T2));
        };
        // CU columns' loads in flight together (P * CU = HGM_MGS1_LD pairs a lane)
#ifndef HGM_MGS1_LD
#define HGM_MGS1_LD 8
#endif
        constexpr int CU = HGM_MGS1_LD / P >= 2 ? HGM_MGS1_LD / P : 2;
        int c = 0;
#pragma unroll 1
        for (; c + CU <= kk + 1; c += CU) {
            T2 qa[CU][P];
#pragma unroll
            for (int u = 0; u < CU; ++u) load(c + u, qa[u]);
#pragma unroll
            for (int u = 0; u < CU; ++u) col(qa[u], c + u);
        }
#pragma unroll 1
        for (; c <= kk; ++c) {
            T2 qa[P];
            load(c, qa);
            col(qa, c);
        }
        if (gx) {                                 // q_k'x_true
            const T2* xt = reinterpret_cast<const T2*>(xe) + tl * tp;
            T a = 0;
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const T2 xx = ok[p] ? xt[ix[p]] : T2{0, 0};
                a = __builtin_fma(qk[p].y, xx.y, __builtin_fma(qk[p].x, xx.x, a));
            }
            add(2 * kk + 2, a);
        }
    }
    __syncthreads();
    if ((n & 1) && b == npr - 1 && t == 0) {      // the odd last element, into wave 0's share
        const int64_t i = n - 1;
        const T wi = w[i];
        const T qki = hpend ? scale(Q[(int64_t)kk * ldq + i]) : Q[(int64_t)kk * ldq + i];
        for (int c2 = 0; c2 <= kk; ++c2) {
            const T qi = (hpend && c2 == kk) ? qki : Q[(int64_t)c2 * ldq + i];
            acc[c2][0] = __builtin_fma(qi, wi, acc[c2][0]);
            if (c2 < kk || gx) acc[kk + 1 + c2][0] = __builtin_fma(qi, qki, acc[kk + 1 + c2][0]);
        }
        if (gx) acc[2 * kk + 2][0] = __builtin_fma(qki, xe[i], acc[2 * kk + 2][0]);
    }
    __syncthreads();
    // rows 0..kk -> pr rows; Gram rows kk+1+c -> pg row c (c = kk: q_k'q_k, c = kk+1: q_k'x_true)
    for (int r = t; r < nrow; r += BS) {
        T v = acc[r][0];
#pragma unroll
        for (int q = 1; q < NW; ++q) v += acc[r][q];
        if (r <= kk) pr[(int64_t)r * npr + b] = v;
        else pg[(int64_t)(r - kk - 1) * npr + b] = v;
    }
}

// The partial rows of k_mgs1_dots reduced exactly as k_mgs1_solve reduces them (16 lanes per
// row, the same loads and additions in the same order, so the same bits), NT threads per block.
template <typename T, int NT>
__device__ __forceinline__ T mgs1_row_sum(const T* p, int npr, bool ok, int sub) {
    T acc = 0;
    for (int base = 0; base < npr; base += 256) {
        T pv[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int i = base + sub + 16 * u;
            pv[u] = (ok && i < npr) ? p[i] : T(0);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += pv[u];
    }
    return row16_sum(acc);
}

// Arguments of the fused form of k_mgs1_update (HGM_OPT_MGS_FUSED): the update blocks run
// k_mgs1_solve's reduction and substitution themselves, redundantly per block, so the sweep is
// two dependent launches (dots, update) instead of three.
template <typename T>
struct Mgs1Fused {
    const T* pr = nullptr;   // partial rows r_0..r_k (npr each)
    const T* pg = nullptr;   // partial rows of the Gram row k (+ q_k'q_k, q_k'x_true)
    int npr = 0;
    T* Gt = nullptr;         // packed Gram triangle kept across the steps (block 0 appends row k)
    int ngx = 0;             // 2: Gram error monitor rows
};

// One 1024-thread workgroup.  MODE 0: sum the partial rows and solve.  MODE 1: sum only,
// red = [r_0..r_k | g_0..g_{k-1}] (multi-GPU all-reduces it).  MODE 2: solve from red.
// Row c < k+1 is r_c (pr), row k+1+c is g_c (pg); 16 lanes (one DPP row) per partial row.
// Gt: the packed strictly lower Gram triangle (row j at j(j-1)/2), kept across the steps
// of a solve (step k appends row k); dynamic LDS holds its k(k+1)/2 values.
constexpr int MGS1_SBS = 1024;
template <typename T, int MODE>
__global__ __launch_bounds__(MGS1_SBS) void k_mgs1_solve(int kk, const T* __restrict__ pr, const T* __restrict__ pg,
                                                         int npr, T* red, T* Gt, T* hdev, T* gx) {
    extern __shared__ unsigned char mgs1_smem[];
    T* sG = reinterpret_cast<T*>(mgs1_smem);
    __shared__ T sr[MGS1_MAXC];
    const int t = threadIdx.x;
    const int rowk = kk * (kk - 1) / 2;   // offset of Gram row kk
    // gx (MODE 0, Gram error monitor): rows 2k+1, 2k+2 = q_k'q_k, q_k'x_true (pg rows k, k+1)
    const int nrow = 2 * kk + 1 + (MODE == 0 && gx ? 2 : 0);
    auto put = [&](int row, T a) {
        if (row <= kk) {
            sr[row] = a;
        } else if (row > 2 * kk) {
            gx[row - 2 * kk - 1] = a;
        } else {
            sG[rowk + row - kk - 1] = a;
            Gt[rowk + row - kk - 1] = a;
        }
    };
    // rows 1..k-1 of the triangle (earlier steps): issued first, independent of the sums
    for (int e = t; e < rowk; e += MGS1_SBS) sG[e] = Gt[e];
    if (MODE != 2) {
        const int sub = t & 15;
        for (int row0 = 0; row0 < nrow; row0 += MGS1_SBS / 16) {
            const int row = row0 + (t >> 4);
            const bool ok = row < nrow;
            const T* p = row <= kk ? pr + (int64_t)row * npr : pg + (int64_t)(row - kk - 1) * npr;
            const T acc = mgs1_row_sum<T, MGS1_SBS>(p, npr, ok, sub);
            if (sub == 0 && ok) {
                if (MODE == 1) red[row] = acc;
                else put(row, acc);
            }
        }
        if (MODE == 1) return;
    } else {
        for (int row = t; row < nrow; row += MGS1_SBS) put(row, red[row]);
    }
    __syncthreads();
    if ((t >> 6) == 0) mgs1_substitute(kk, sr, sG, hdev);
}

template <typename T, bool FUSED, int P>
// hpend: Q(:,k) still holds v_k (pending normalisation): q_k = v_k / *hpend is used for the
// last term and written back (each element by the one thread that updates it).
// (4 waves per SIMD: the 1024-block cap is resident at once)
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(4))) void k_mgs1_update(int64_t n, int nb, T* Q, int64_t ldq, int kk,
                                                    const T* w, T* v, const T* __restrict__ hdev, T* Hcol,
                                                    T* __restrict__ pout, MdotStage<T> side, const T* hpend,
                                                    const T* __restrict__ grow, const T* __restrict__ gx, T* qg,
                                                    Mgs1Fused<T> fz) {
    using T2 = typename V2<T>::t;
    __shared__ T hs[MGS1_MAXC];
    __shared__ T sh[4];
    if ((int)blockIdx.x >= nb) {
        mdot_side(side, (int)blockIdx.x - nb, sh);
        return;
    }
    if (FUSED) {
        extern __shared__ unsigned char mgs1u_smem[];
        T* sG = reinterpret_cast<T*>(mgs1u_smem);
        __shared__ T sr[MGS1_MAXC];
        __shared__ T sgx[2];
        const int t = threadIdx.x, sub = t & 15;
        const int rowk = kk * (kk - 1) / 2;
        const int nrow = 2 * kk + 1 + fz.ngx;
        for (int e = t; e < rowk; e += BS) sG[e] = fz.Gt[e];
        for (int row0 = 0; row0 < nrow; row0 += BS / 16) {
            const int row = row0 + (t >> 4);
            const bool ok = row < nrow;
            const T* p = row <= kk ? fz.pr + (int64_t)row * fz.npr : fz.pg + (int64_t)(row - kk - 1) * fz.npr;
            const T acc = mgs1_row_sum<T, BS>(p, fz.npr, ok, sub);
            if (sub == 0 && ok) {
                if (row <= kk) {
                    sr[row] = acc;
                } else if (row > 2 * kk) {
                    sgx[row - 2 * kk - 1] = acc;
                } else {
                    sG[rowk + row - kk - 1] = acc;
                    if (blockIdx.x == 0) fz.Gt[rowk + row - kk - 1] = acc;
                }
            }
        }
        __syncthreads();
        if ((t >> 6) == 0) mgs1_substitute(kk, sr, sG, hs);
        __syncthreads();
        if (blockIdx.x == 0) {
            for (int j = t; j <= kk; j += BS) st_sys(Hcol + j, hs[j]);   // H(0:k, k) -> host ring
            if (qg)                                                      // Gram error monitor row
                for (int j = t; j <= kk + 1; j += BS) st_sys(qg + j, j < kk ? sG[rowk + j] : sgx[j - kk]);
        }
    } else {
        for (int j = threadIdx.x; j <= kk; j += BS) {
            const T h = hdev[j];
            hs[j] = h;
            if (blockIdx.x == 0) st_sys(Hcol + j, h);   // H(0:k, k) -> host ring
        }
        if (qg && blockIdx.x == 0)                      // Gram error monitor row -> host ring
            for (int j = threadIdx.x; j <= kk + 1; j += BS) st_sys(qg + j, j < kk ? grow[j] : gx[j - kk]);
        __syncthreads();
    }
    const int64_t n2 = n >> 1, stride = (int64_t)nb * BS;
    const T2* w2 = reinterpret_cast<const T2*>(w);
    T2* v2 = reinterpret_cast<T2*>(v);
    const T hp = hpend ? *hpend : T(0);
    auto scale = [&](T x) -> T { return hp != T(0) ? x / hp : x; };   // as k_mgs_normalize
    const int jn = hpend ? kk : kk + 1;                               // columns read as stored
    T2* qk2 = reinterpret_cast<T2*>(Q + (int64_t)kk * ldq);
    T acc0 = 0, acc1 = 0;
    // Tiles of BS*P element pairs per block, swept column by column (CW columns' loads in flight
    // at a time): a block streams a few columns at a time instead of touching all k+3 vectors
    // per element (C3 at k = 19: 4.6 TB/s that way, against 6 TB/s at k = 5).  Every element's
    // subtraction order is MGS's, j = 0..k.
    constexpr int CW = 16 / P;                         // (16 pairs a lane in flight)
    const int64_t tp = (int64_t)BS * P, ntile = (n2 + tp - 1) / tp;
    (void)stride;
    for (int64_t tl = blockIdx.x; tl < ntile; tl += nb) {
        const T2* wt = w2 + tl * tp;
        const int lim = (int)min<int64_t>(tp, n2 - tl * tp);   // pairs in this tile
        int ix[P];
        T2 vv[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const int e = (int)threadIdx.x + p * BS;
            ix[p] = e < lim ? e : lim - 1;            // (past the end: a repeated load, not stored)
            vv[p] = wt[ix[p]];
        }
        auto sub = [&](const T2* qq, T h) {
#pragma unroll
            for (int p = 0; p < P; ++p) {
                const T p0 = h * qq[p].x, p1 = h * qq[p].y;
                vv[p].x = vv[p].x - p0;
                vv[p].y = vv[p].y - p1;
            }
        };
        // (buffer loads: one 32-bit offset per pair serves every column, a scalar base per column)
        const T2* qt = reinterpret_cast<const T2*>(Q) + tl * tp;
        const int64_t ld2 = ldq >> 1;                 // (ldq is even: a multiple of 64)
        auto col = [&](int jj) { return buf_rsrc(qt + (int64_t)jj * ld2, lim * (int)sizeof(T2)); };
        int j = 0;
#pragma unroll 1
        for (; j + CW <= jn; j += CW) {
            T2 r[CW][P];
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                const __amdgpu_buffer_rsrc_t rc = col(j + c);
#pragma unroll
                for (int p = 0; p < P; ++p) r[c][p] = buf_load2<T2>(rc, ix[p] * (int)sizeof(T2));
            }
#pragma unroll
            for (int c = 0; c < CW; ++c) sub(r[c], hs[j + c]);
        }
#pragma unroll 1
        for (; j < jn; ++j) {
            T2 r[P];
            const __amdgpu_buffer_rsrc_t rc = col(j);
#pragma unroll
            for (int p = 0; p < P; ++p) r[p] = buf_load2<T2>(rc, ix[p] * (int)sizeof(T2));
            sub(r, hs[j]);
        }
        if (hpend) {                                  // q_k = v_k / H(k,k-1), written back
            T2* qkt = qk2 + tl * tp;
            T2 r[P];
#pragma unroll
            for (int p = 0; p < P; ++p) {
                r[p] = qkt[ix[p]];
                r[p].x = scale(r[p].x);
                r[p].y = scale(r[p].y);
            }
#pragma unroll
            for (int p = 0; p < P; ++p)
                if ((int)threadIdx.x + p * BS < lim) qkt[ix[p]] = r[p];
            sub(r, hs[kk]);
        }
        T2* vt = v2 + tl * tp;
#pragma unroll
        for (int p = 0; p < P; ++p)
            if ((int)threadIdx.x + p * BS < lim) {
                vt[ix[p]] = vv[p];
                acc0 += vv[p].x * vv[p].x;
                acc1 += vv[p].y * vv[p].y;
            }
    }
    if ((n & 1) && (int)blockIdx.x == nb - 1 && threadIdx.x == 0) {
        const int64_t i = n - 1;
        T vv = w[i];
        T qkk = 0;
        if (hpend) {
            qkk = scale(Q[(int64_t)kk * ldq + i]);
            Q[(int64_t)kk * ldq + i] = qkk;
        }
        for (int j = 0; j <= kk; ++j) {
            const T p = hs[j] * ((j == kk && hpend) ? qkk : Q[(int64_t)j * ldq + i]);
            vv = vv - p;
        }
        v[i] = vv;
        acc0 += vv * vv;
    }
    const T tot = block_sum_all<T, false>(acc0 + acc1, sh);
    if (threadIdx.x == 0) pout[blockIdx.x] = tot;
}

// ------------------------------------------------------------------------------
// MGS in parity mode (HGM_OPT_PARITY): hybrid_ba_gmres_rtp.m:20-26 as written, one
// fixed-order dot and one axpy launch per column:
//   h_j = Q(:,j)'v (fixed order) ; v = v - h_j Q(:,j) (two roundings) ; H(k+1,k) = norm(v) ;
//   Q(:,k+1) = v / H(k+1,k) unless H(k+1,k) == 0
// ------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(BS) void k_axpy_hdev(int64_t n, T* v, const T* src, const T* __restrict__ q,
                                                  const T* hp) {
    const T h = *hp;
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
        const T p = h * q[i];
        v[i] = src[i] - p;
    }
}
// hd[kk+1] = sqrt(hd[kk+1]) (the fixed-order sum of squares), H(0:kk+1,kk) -> Hcol (system-scope
// stores: Hcol may be the host ring), then v = v / H(kk+1,kk) unless it is zero
template <typename T>
__global__ __launch_bounds__(BS) void k_mgs_parity_fin(int64_t n, int kk, T* v, const T* hd, T* Hcol) {
    const T nrm = sqrt(hd[kk + 1]);
    if (blockIdx.x == 0)
        for (int j = threadIdx.x; j <= kk + 1; j += BS) st_sys(Hcol + j, j <= kk ? hd[j] : nrm);
    if (nrm == T(0)) return;
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) v[i] = v[i] / nrm;
}

template <typename T>
static void mgs_parity(hgm_ctx* c, int64_t n, T* Q, int64_t ldq, int kk, T* Hcol, const T* src) {
    T* v = Q + (int64_t)(kk + 1) * ldq;
    T* hd = c->buf<T>("mgsp_h", kk + 3);
    const int g = grid_for(n);
    const T* cur = src;
    for (int j = 0; j <= kk; ++j) {
        const T* qj = Q + (int64_t)j * ldq;
        fixed_reduce_op<T, 0>(c, n, qj, cur, 0, nullptr, nullptr, hd + j);   // :21  H(j,k) = Q(:,j)'*v
        k_axpy_hdev<T><<<g, BS, 0, c->stream>>>(n, v, cur, qj, hd + j);       // :22  v = v - H(j,k)*Q(:,j)
        cur = v;
    }
    fixed_reduce_op<T, 1>(c, n, v, v, 0, nullptr, nullptr, hd + kk + 1);      // :24  H(k+1,k) = norm(v)
    k_mgs_parity_fin<T><<<g, BS, 0, c->stream>>>(n, kk, v, hd, Hcol);         // :26  Q(:,k+1) = v / H(k+1,k)
    HGM_HIP(hipGetLastError());
}

template <typename T>
void mgs(hgm_ctx* c, int64_t n, T* Q, int64_t ldq, int kk, T* Hcol, bool dist, const T* src,
         const MdotJob<T>* side, PendNorm<T>* defer, const T* pend_h, const T* xe, T* qg, const double* cp_src,
         double* cp_dst) {
    if (defer) defer->np = 0;
    // the ring copy rides on the one-reduction sweep's dots kernel; every other form copies first
    const int64_t sq = ldq / MGS1_BS;   // (mgs_single's shapes)
    const bool single = !dist && krylov_padded(c, ldq) && n <= ldq && sq % 4 == 0 && sq >= 4 && sq <= 24;
    if (cp_dst && !(kk + 1 <= MGS1_MAXC && mgs1_mode(c) == 1 && !c->num.parity && !single)) {
        copy_sys(c, cp_src, cp_dst);
        cp_dst = nullptr;
    }
    if (c->num.parity) {
        HGM_REQUIRE(!dist && !xe && !pend_h, "mgs: parity mode is single-rank, without the fused monitors");
        hipEvent_t t0 = nullptr;
        timing_begin(c, KC_MGS, &t0);
        mgs_parity<T>(c, n, Q, ldq, kk, Hcol, src ? src : Q + (int64_t)(kk + 1) * ldq);
        if (side) multidot<T>(c, side->n, side->ncols, side->Q, side->ldq, side->w, side->out, side->e);
        timing_end(c, KC_MGS, t0, sizeof(T) * (double)n * (4.0 * kk + 7.0));
        return;
    }
    HGM_REQUIRE(!xe || (qg && !dist && kk + 1 <= MGS1_MAXC && mgs1_mode(c) == 1 && !krylov_padded(c, ldq)),
                "mgs: the Gram error monitor needs the one-reduction form");
    HGM_REQUIRE(!pend_h || (!dist && kk + 1 <= MGS1_MAXC && mgs1_mode(c) == 1 && !krylov_padded(c, ldq)),
                "mgs: pending normalisation needs the one-reduction form");
    hipEvent_t t0 = nullptr;
    timing_begin(c, KC_MGS, &t0);
    const double s = sizeof(T);
    T* v = Q + (int64_t)(kk + 1) * ldq;
    if (src == nullptr) src = v;
    if (!dist && mgs_single<T>(c, n, Q, ldq, kk, Hcol, src)) {
        timing_end(c, KC_MGS, t0, s * n * (kk + 3.0));   // q_0..q_kk and v read once, v written once
        if (side) multidot<T>(c, side->n, side->ncols, side->Q, side->ldq, side->w, side->out, side->e);
        return;
    }
    if (kk + 1 <= MGS1_MAXC && mgs1_mode(c) == 1) {
        MdotStage<T> s1, s2;
        if (side && !dist) {
            s1.j = *side;
            s1.np = parts_for(side->n);
            s1.parts = c->buf<T>("mdot_parts", (size_t)s1.np * (side->ncols + 1));
            s1.stage = 1;
            s2 = s1;
            s2.stage = 2;
        }
        hipStream_t st = c->stream;
        const int P = mgs1_tile(c, n);
        const int npr = mgs1_blocks(n, P);
        T* pr = c->buf<T>("mgs1_pr", (size_t)MGS1_MAXC * MAX_PARTS);
        T* pg = c->buf<T>("mgs1_pg", (size_t)(MGS1_MAXC + 2) * MAX_PARTS);
        T* gx = xe ? c->buf<T>("mgs1_gx", 2) : nullptr;
        T* Gt = c->buf<T>("mgs1_G", (size_t)MGS1_MAXC * MGS1_MAXC / 2 + MGS1_MAXC);
        T* hdev = c->buf<T>("mgs1_h", MGS1_MAXC + 2);
        const size_t lds = sizeof(T) * ((size_t)kk * (kk + 1) / 2 + 1);
#define HGM_MGS1_P(PV, STMT) \
    if (P == PV) {          \
        constexpr int PT = PV; \
        STMT;               \
    }
#define HGM_MGS1_PS(STMT) HGM_MGS1_P(1, STMT) else HGM_MGS1_P(2, STMT) else HGM_MGS1_P(4, STMT) else HGM_REQUIRE(false, "mgs1: tile width")
        HGM_MGS1_PS((k_mgs1_dots<T, PT><<<npr + s1.blocks(), BS, 0, st>>>(n, Q, ldq, kk, src, npr, pr, pg, s1, pend_h, xe,
                                                                          cp_src, cp_dst)));
        const int nb = npr;
        T* pout = c->buf<T>("mgs_parts", 2 * MAX_PARTS);
        const bool fused = !dist && c->num.mgs_fused;
        Mgs1Fused<T> fz;
        if (fused) {
            fz.pr = pr;
            fz.pg = pg;
            fz.npr = npr;
            fz.Gt = Gt;
            fz.ngx = xe ? 2 : 0;
            HGM_MGS1_PS((k_mgs1_update<T, true, PT><<<nb + s2.blocks(), BS, lds, st>>>(
                n, nb, Q, ldq, kk, src, v, hdev, Hcol, pout, s2, pend_h, nullptr, nullptr, xe ? qg : nullptr, fz)));
        } else if (dist) {
            T* redd = c->buf<T>("mgs1_red", 2 * MGS1_MAXC + 2);
            k_mgs1_solve<T, 1><<<1, MGS1_SBS, 0, st>>>(kk, pr, pg, npr, redd, Gt, hdev, nullptr);
            allreduce(c, redd, 2 * kk + 1);
            k_mgs1_solve<T, 2><<<1, MGS1_SBS, lds, st>>>(kk, pr, pg, npr, redd, Gt, hdev, nullptr);
        } else {
            k_mgs1_solve<T, 0><<<1, MGS1_SBS, lds, st>>>(kk, pr, pg, npr, nullptr, Gt, hdev, gx);
        }
        if (!fused) {
            HGM_MGS1_PS((k_mgs1_update<T, false, PT><<<nb + s2.blocks(), BS, 0, st>>>(
                n, nb, Q, ldq, kk, src, v, hdev, Hcol, pout, s2, pend_h, Gt + (size_t)kk * (kk - 1) / 2, gx,
                xe ? qg : nullptr, fz)));
        }
#undef HGM_MGS1_PS
#undef HGM_MGS1_P
        if (defer && !dist && kk + 2 <= MGS1_MAXC) {   // the next step must be one-reduction too
            // the next step's SpMVs divide by H(kk+1,kk) in their epilogues
            HGM_HIP(hipGetLastError());
            defer->parts = pout;
            defer->np = nb;
            timing_end(c, KC_MGS, t0, s * n * (2.0 * kk + 6.0));
            return;
        }
        T* ss = c->buf<T>("mgs_ss", 4);
        if (dist) {
            k_finalize<T><<<1, BS, 0, st>>>(pout, nb, ss);
            allreduce(c, ss, 1);
        }
        k_mgs_normalize<T><<<nb, BS, 0, st>>>(n, v, pout, dist ? 0 : nb, ss, Hcol + kk + 1);
        HGM_HIP(hipGetLastError());
        if (side && dist) multidot<T>(c, side->n, side->ncols, side->Q, side->ldq, side->w, side->out, side->e);
        // dots read w and q_0..q_k (+ q_k per column group), the update reads w and
        // q_0..q_k and writes v, the scale reads and writes v
        timing_end(c, KC_MGS, t0, s * n * (2.0 * kk + 8.0));
        return;
    }
    // the side multidot rides on passes 0 and 1 (single GPU; with ranks it keeps its own
    // launches after the sweep, whose passes are separated by all-reduces)
    MdotStage<T> s1, s2, none;
    if (side && !dist) {
        s1.j = *side;
        s1.np = parts_for(side->n);
        s1.parts = c->buf<T>("mdot_parts", (size_t)s1.np * (side->ncols + 1));
        s1.stage = 1;
        s2 = s1;
        s2.stage = 2;
    }
    // One launch per pass: a dependent launch is the cheapest grid-wide exchange of the
    // block partials on gfx950 (2.6-2.9 us vs 3-25 us for in-kernel grid barriers,
    // scripts/barrier_bench.hip).
    const int np = gemv_blocks(n, mgs_ppl(c));
    T* P = c->buf<T>("mgs_parts", 2 * MAX_PARTS);
    T* Pb[2] = {P, P + MAX_PARTS};
    T* ss = c->buf<T>("mgs_ss", 4);
    hipStream_t st = c->stream;
    // pass 0: h_0 partials
    k_mgs_pass<T, 0><<<np + s1.blocks(), BS, 0, st>>>(n, np, nullptr, Q, src, v, nullptr, 0, nullptr, nullptr,
                                                       Pb[0], s1);
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
            const MdotStage<T>& sj = j == 1 ? s2 : none;
            k_mgs_pass<T, 1><<<np + sj.blocks(), BS, 0, st>>>(n, np, qa, qd, j == 1 ? src : v, v, pin, np_in,
                                                               Hcol + (j - 1), hdst, pout, sj);
            if (dist) {
                k_finalize<T><<<1, BS, 0, st>>>(pout, np, Hcol + j);
                allreduce(c, Hcol + j, 1);
            }
        } else {
            const MdotStage<T>& sj = j == 1 ? s2 : none;
            k_mgs_pass<T, 2><<<np + sj.blocks(), BS, 0, st>>>(n, np, qa, nullptr, j == 1 ? src : v, v, pin, np_in,
                                                               Hcol + (j - 1), hdst, pout, sj);
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
    if (side && dist) multidot<T>(c, side->n, side->ncols, side->Q, side->ldq, side->w, side->out, side->e);
    // algorithmic bytes: (32k+24)n-style count for k+1 = kk+1 columns
    const double bytes = s * n * (2.0 + 4.0 * kk + 3.0 + 2.0);
    timing_end(c, KC_MGS, t0, bytes);
}

template <typename T>
void gemv(hgm_ctx* c, int64_t n, int k, const T* Q, int64_t ldq, const T* y, T* x, int mode) {
    HGM_REQUIRE(k <= GEMV_KMAX && ldq % 2 == 0, "gemv: k too large");
    const int nb = gemv_blocks(n);
    const size_t sm = sizeof(T) * (k > 0 ? k : 1);
    if (mode == 0) k_gemv2<T, 0, false><<<nb, BS, sm, c->stream>>>(n, k, Q, ldq, y, x, nullptr, nullptr);
    else k_gemv2<T, 1, false><<<nb, BS, sm, c->stream>>>(n, k, Q, ldq, y, x, nullptr, nullptr);
    HGM_HIP(hipGetLastError());
}

// Classical Gram-Schmidt applied twice (option; C3's MGS vs CGS2 comparison).
template <typename T>
__global__ __launch_bounds__(BS) void k_add_store(int k, const T* a, const T* b, T* out) {
    const int i = threadIdx.x;
    if (i < k) st_sys(out + i, a[i] + b[i]);
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

// v = v / sqrt(sum parts) (every block re-reduces the partials in the fixed order of
// k_finalize); block 0 stores the norm to *nrm_out with a system-scope store.  Divides even by
// a zero norm, as MATLAB's r0 / beta does.
template <typename T>
__global__ __launch_bounds__(BS) void k_vnorm(int64_t n, T* __restrict__ v, const T* __restrict__ parts, int np,
                                              T* nrm_out) {
    __shared__ T sh[4];
    const T nrm = sqrt(reduce_parts<T, false>(parts, np, sh));
    if (blockIdx.x == 0 && threadIdx.x == 0) st_sys(nrm_out, nrm);
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) v[i] = v[i] / nrm;
}
// parity mode: v = v / sqrt(*ss) (*ss from a fixed-order sum), norm stored to *nrm_out
template <typename T>
__global__ __launch_bounds__(BS) void k_vnorm_ss(int64_t n, T* __restrict__ v, const T* ss, T* nrm_out) {
    const T nrm = sqrt(*ss);
    if (blockIdx.x == 0 && threadIdx.x == 0) st_sys(nrm_out, nrm);
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) v[i] = v[i] / nrm;
}
template <typename T> void normalize_to(hgm_ctx* c, int64_t n, T* v, T* nrm_out) {
    if (c->num.parity) {
        T* ss = c->buf<T>("vnorm_ss", 2);
        fixed_reduce_op<T, 1>(c, n, v, v, 0, nullptr, nullptr, ss);
        k_vnorm_ss<T><<<grid_for(n), BS, 0, c->stream>>>(n, v, ss, nrm_out);
        HGM_HIP(hipGetLastError());
        return;
    }
    const int np = parts_for(n);
    T* parts = c->buf<T>("red_parts", MAX_PARTS);
    if (al16(v)) k_reduce_partial<T, 1, true><<<np, BS, 0, c->stream>>>(n, v, v, parts);
    else k_reduce_partial<T, 1, false><<<np, BS, 0, c->stream>>>(n, v, v, parts);
    k_vnorm<T><<<grid_for(n), BS, 0, c->stream>>>(n, v, parts, np, nrm_out);
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

// ------------------------------------------------------------------------------
// Device-resident LSQR scalars (lsqr_solver.m:22-46 without host round trips): the Givens
// rotation of :31-38 in one thread, in double, exactly as the host loop computes it from the
// same sums of squares, and the stop test of :44-46 as a flag the update kernel honours.
// st: [rho_bar, phi_bar, stop] (stop = iteration+1 of the first res <= tol, 0 while running).
// ------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void scalar_copies(const ScalarCopy<T>& cp) {
    if (cp.dst) *cp.dst = *cp.src;
    if (cp.ddst) *cp.ddst = *cp.dsrc;
}
template <typename T>
__global__ void k_copy_scalars(ScalarCopy<T> cp) {
    if (threadIdx.x == 0 && blockIdx.x == 0) scalar_copies(cp);
}
template <typename T>
void copy_scalars(hgm_ctx* c, const ScalarCopy<T>& cp) {
    k_copy_scalars<T><<<1, 64, 0, c->stream>>>(cp);
    HGM_HIP(hipGetLastError());
}
template void copy_scalars<double>(hgm_ctx*, const ScalarCopy<double>&);
template void copy_scalars<float>(hgm_ctx*, const ScalarCopy<float>&);

template <typename T>
__global__ void k_lsqr_rot(const T* ssb, const T* ssa, double* st, T* coef, double* phib_hist, int k, double nb,
                           double tol, ScalarCopy<T> cp) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    scalar_copies(cp);
    const double beta = sqrt((double)*ssb);                  // :23
    const double alpha = sqrt((double)*ssa);                 // :27
    const double rho_bar = st[0], phi_bar = st[1];
    const double rho = sqrt(rho_bar * rho_bar + beta * beta);   // :31
    const double cs = rho_bar / rho;                         // :32
    const double sn = beta / rho;                            // :33
    const double theta = sn * alpha;                         // :34
    st[0] = -cs * alpha;                                     // :35
    const double phi = cs * phi_bar;                         // :37
    const double pb = sn * phi_bar;                          // :38
    st[1] = pb;
    coef[0] = (T)(phi / rho);                                // :40
    coef[1] = (T)(theta / rho);                              // :41
    phib_hist[k] = pb;
    if (st[2] == 0.0 && fabs(pb) / nb <= tol) st[2] = (double)(k + 1);   // :44-46
}

// v = v_hat / alpha (alpha = sqrt(*ssa)), then x += (phi/rho) w ; w = v - (theta/rho) w
// (lsqr_solver.m:28,40-41), skipped once an earlier iteration met the stop test; with parts,
// also the partials of ||x - x_true||^2 (:43) in k_reduce_partial<T, 2>'s order (same bits).
template <typename T, bool VEC>
__global__ __launch_bounds__(BS) void k_lsqr_step(int64_t n, T* __restrict__ x, T* __restrict__ w, T* __restrict__ v,
                                                  const T* ssa, const T* coef, const double* st, int k,
                                                  const T* __restrict__ xt, T* __restrict__ parts) {
    __shared__ T sh[4];
    const T alpha = (T)sqrt((double)*ssa);
    const bool live = !(st[2] != 0.0 && st[2] < (double)(k + 1));
    const T a = coef[0], b = coef[1];
    T acc = 0;
    grid_elems<T, VEC>(n, [&](int64_t i, auto wc) {
        constexpr int W = decltype(wc)::value;
        T vv[W], xx[W], ww[W], tt[W];
        vload<W>(v, i, vv);
        vload<W>(x, i, xx);
        if (live) vload<W>(w, i, ww);
        if (parts) vload<W>(xt, i, tt);
#pragma unroll
        for (int e = 0; e < W; ++e) {
            vv[e] = vv[e] / alpha;
            if (live) {
                const T p = a * ww[e];
                xx[e] = xx[e] + p;
                const T q = b * ww[e];
                ww[e] = vv[e] - q;
            }
            if (parts) {
                const T d = xx[e] - tt[e];
                acc += d * d;
            }
        }
        vstore<W>(v, i, vv);
        if (live) {
            vstore<W>(x, i, xx);
            vstore<W>(w, i, ww);
        }
    });
    if (parts) {
        const T tot = block_sum_all(acc, sh);
        if (threadIdx.x == 0) parts[blockIdx.x] = tot;
    }
}

// out = in / (T)sqrt((double)*ss)
template <typename T>
__global__ __launch_bounds__(BS) void k_div_sqrt(int64_t n, const T* __restrict__ in, T* __restrict__ out, const T* ss) {
    const T s = (T)sqrt((double)*ss);
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) out[i] = in[i] / s;
}

template <typename T>
void lsqr_rot(hgm_ctx* c, const T* ssb, const T* ssa, double* st, T* coef, double* phib_hist, int k, double nb,
              double tol, const ScalarCopy<T>& cp) {
    k_lsqr_rot<T><<<1, 64, 0, c->stream>>>(ssb, ssa, st, coef, phib_hist, k, nb, tol, cp);
    HGM_HIP(hipGetLastError());
}

template <typename T>
void lsqr_step(hgm_ctx* c, int64_t n, T* x, T* w, T* v, const T* ssa, const T* coef, const double* st, int k,
               const T* xt, T* err_out) {
    // the error partials keep reduce_to's layout: one launch for short vectors stays separate
    const bool fuse = xt && n > SINGLE_MAX && !c->num.parity;
    const int np = fuse ? parts_for(n) : grid_for(n);
    T* parts = fuse ? c->buf<T>("red_parts", MAX_PARTS) : nullptr;
    // (vectors as k_reduce_partial takes them for the same x and x_true: the same error bits)
    if (al16(x) && al16(w) && al16(v) && (!xt || al16(xt)))
        k_lsqr_step<T, true><<<np, BS, 0, c->stream>>>(n, x, w, v, ssa, coef, st, k, xt, parts);
    else
        k_lsqr_step<T, false><<<np, BS, 0, c->stream>>>(n, x, w, v, ssa, coef, st, k, xt, parts);
    if (fuse) k_finalize<T><<<1, BS, 0, c->stream>>>(parts, np, err_out);
    HGM_HIP(hipGetLastError());
    if (xt && !fuse) sumsq_diff<T>(c, n, x, xt, err_out);
}

template <typename T>
void div_sqrt(hgm_ctx* c, int64_t n, const T* in, T* out, const T* ss) {
    k_div_sqrt<T><<<grid_for(n), BS, 0, c->stream>>>(n, in, out, ss);
    HGM_HIP(hipGetLastError());
}

// The m-space half of a Golub-Kahan step after the one-pass w = A*(A'*u - beta*v) (fused.hip):
// A*v_k = w / alpha_k (alpha = (T)sqrt((double)*ssa); a zero alpha leaves w, as lsmr_solver.m:16/40
// leave v undivided), kept in av when given, then t = A*v_k - alpha*u (lsqr_solver.m:22,
// lsmr_solver.m:34; two roundings, as the two-pass EPI_SUB epilogue), with the partials of ||t||^2
// in k_reduce_partial<T, 1>'s layout (parts == nullptr: none).
template <typename T, bool VEC>
__global__ __launch_bounds__(BS) void k_gkb_mstep(int64_t n, const T* __restrict__ w, const T* ssa,
                                                  const T* __restrict__ u, T* __restrict__ t, T* __restrict__ av,
                                                  T* __restrict__ parts) {
    __shared__ T sh[4];
    const T a = (T)sqrt((double)*ssa);
    T acc = 0;
    grid_elems<T, VEC>(n, [&](int64_t i, auto wc) {
        constexpr int W = decltype(wc)::value;
        T ww[W], uu[W], tt[W];
        vload<W>(w, i, ww);
        vload<W>(u, i, uu);
#pragma unroll
        for (int e = 0; e < W; ++e) {
            ww[e] = a != T(0) ? ww[e] / a : ww[e];
            const T s = a * uu[e];
            tt[e] = ww[e] - s;
            acc += tt[e] * tt[e];
        }
        if (av) vstore<W>(av, i, ww);
        vstore<W>(t, i, tt);
    });
    if (parts) {
        const T tot = block_sum_all(acc, sh);
        if (threadIdx.x == 0) parts[blockIdx.x] = tot;
    }
}

template <typename T>
void gkb_mstep(hgm_ctx* c, int64_t n, const T* w, const T* ssa, const T* u, T* t, T* av, T* ss_out) {
    const bool fuse = n > SINGLE_MAX && !c->num.parity;
    const int np = fuse ? parts_for(n) : grid_for(n);
    T* parts = fuse ? c->buf<T>("red_parts", MAX_PARTS) : nullptr;
    if (al16(w) && al16(u) && al16(t) && (!av || al16(av)))
        k_gkb_mstep<T, true><<<np, BS, 0, c->stream>>>(n, w, ssa, u, t, av, parts);
    else
        k_gkb_mstep<T, false><<<np, BS, 0, c->stream>>>(n, w, ssa, u, t, av, parts);
    if (fuse) k_finalize<T><<<1, BS, 0, c->stream>>>(parts, np, ss_out);
    HGM_HIP(hipGetLastError());
    if (!fuse) sumsq<T>(c, n, t, ss_out);
}
template void gkb_mstep<double>(hgm_ctx*, int64_t, const double*, const double*, const double*, double*, double*,
                                double*);

// out = in / s with s = (T)sqrt(ss), ss the sum of the np partials of ||in||^2 that every block
// re-forms in k_finalize's order (reduce_parts: the same bits); block 0 publishes ss to ss_out.
// NZ: a zero s leaves in (lsmr_solver.m:36, as k_div_sqrt_nz).  Round 6: replaces the
// k_finalize + k_div_sqrt launch pair of the one-pass Golub-Kahan m-space step.
template <typename T, bool NZ>
__global__ __launch_bounds__(BS) void k_div_sqrt_parts(int64_t n, const T* __restrict__ in, T* __restrict__ out,
                                                       const T* __restrict__ parts, int np, T* ss_out) {
    __shared__ T sh[4];
    const T ssv = reduce_parts(parts, np, sh);
    if (blockIdx.x == 0 && threadIdx.x == 0) st_sys(ss_out, ssv);
    const T s = (T)sqrt((double)ssv);
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
        out[i] = (!NZ || s > T(0)) ? in[i] / s : in[i];
}

// gkb_mstep (t = A*v_k - alpha*u, ||t||^2 -> ss_out) followed by u = t / sqrt(||t||^2) (NZ: as
// div_sqrt_nz): two launches where the separate calls take three (the same bits).
template <typename T>
void gkb_mstep_div(hgm_ctx* c, int64_t n, const T* w, const T* ssa, T* u, T* t, T* av, T* ss_out, bool nz) {
    const bool fuse = n > SINGLE_MAX && !c->num.parity;
    if (!fuse) {
        gkb_mstep<T>(c, n, w, ssa, u, t, av, ss_out);
        if (nz) div_sqrt_nz<T>(c, n, t, u, ss_out);
        else div_sqrt<T>(c, n, t, u, ss_out);
        return;
    }
    const int np = parts_for(n);
    T* parts = c->buf<T>("red_parts", MAX_PARTS);
    if (al16(w) && al16(u) && al16(t) && (!av || al16(av)))
        k_gkb_mstep<T, true><<<np, BS, 0, c->stream>>>(n, w, ssa, u, t, av, parts);
    else
        k_gkb_mstep<T, false><<<np, BS, 0, c->stream>>>(n, w, ssa, u, t, av, parts);
    if (nz) k_div_sqrt_parts<T, true><<<grid_for(n), BS, 0, c->stream>>>(n, t, u, parts, np, ss_out);
    else k_div_sqrt_parts<T, false><<<grid_for(n), BS, 0, c->stream>>>(n, t, u, parts, np, ss_out);
    HGM_HIP(hipGetLastError());
}
template void gkb_mstep_div<double>(hgm_ctx*, int64_t, const double*, const double*, double*, double*, double*,
                                    double*, bool);
template void gkb_mstep_div<float>(hgm_ctx*, int64_t, const float*, const float*, float*, float*, float*, float*,
                                   bool);
template void gkb_mstep<float>(hgm_ctx*, int64_t, const float*, const float*, const float*, float*, float*, float*);

// (one-pass LSQR) the images of x and w under A, in double, so the exact final residual of
// lsqr_solver.m:52 needs no SpMV: with A*v_{k+1} = w_m / alpha_{k+1} (the pass's A*v_hat),
// A*x += (phi/rho) A*w ; A*w = A*v_{k+1} - (theta/rho) A*w (:40-41 under A).  init: A*w = A*v_0,
// A*x = 0.  Iterations enqueued past a device stop (st[2], as k_lsqr_step) change nothing.
template <typename T>
__global__ __launch_bounds__(BS) void k_lsqr_img(int64_t m, const T* __restrict__ wm, const T* ssa, const T* coef,
                                                 const double* st, int k, double* __restrict__ ax,
                                                 double* __restrict__ aw, int init) {
    const double a = (double)(T)sqrt((double)*ssa);
    const bool live = init || !(st[2] != 0.0 && st[2] < (double)(k + 1));
    if (!live) return;
    const double c0 = init ? 0.0 : (double)coef[0], c1 = init ? 0.0 : (double)coef[1];
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < m; i += (int64_t)gridDim.x * BS) {
        const double av = a != 0.0 ? (double)wm[i] / a : (double)wm[i];
        if (init) {
            ax[i] = 0.0;
            aw[i] = av;
        } else {
            ax[i] = ax[i] + c0 * aw[i];
            aw[i] = av - c1 * aw[i];
        }
    }
}
template <typename T>
void lsqr_img(hgm_ctx* c, int64_t m, const T* wm, const T* ssa, const T* coef, const double* st, int k, double* ax,
              double* aw, bool init) {
    k_lsqr_img<T><<<grid_for(m), BS, 0, c->stream>>>(m, wm, ssa, coef, st, k, ax, aw, init ? 1 : 0);
    HGM_HIP(hipGetLastError());
}
template void lsqr_img<double>(hgm_ctx*, int64_t, const double*, const double*, const double*, const double*, int,
                               double*, double*, bool);
template void lsqr_img<float>(hgm_ctx*, int64_t, const float*, const float*, const float*, const double*, int,
                              double*, double*, bool);

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

// Device-resident LSMR scalars (lsmr_solver.m:42-67), the host loop's double arithmetic in one
// thread.  st = [alpha, alphabar, rho, rhobar, cbar, sbar, zetabar, prev (theta/rho), stop];
// *ssb = beta^2, *ssa = alpha^2 of this step.  coef = (T)[c_hbar, c_x, c_h] of :64/:66/:67 for the
// n-space update; cfm / cfn = the monitors' coefficients [c1, c0, f, e, cx] (m-space: image of
// v = A*v_k; n-space: beta A'u_{k+1} + alpha_k A'u_k).
template <typename T>
__global__ void k_lsmr_rot(const T* ssb, const T* ssa, double* st, T* coef, double* cfm, double* cfn,
                           ScalarCopy<T> cp) {
    if (threadIdx.x != 0) return;
    scalar_copies(cp);
    const double alpha_k = st[0];
    const double beta = sqrt((double)*ssb), alpha = sqrt((double)*ssa);   // :35, :39
    const double alphahat = st[1];                                        // :42
    const double rhoold = st[2];                                          // :43
    const double rho = hypot(alphahat, beta);                             // :44
    const double cc = alphahat / rho, ss = beta / rho;                    // :45-46
    const double thetanew = ss * alpha;                                   // :48
    st[1] = cc * alpha;                                                   // :49 alphabar
    const double rhobarold = st[3];                                       // :51
    const double thetabar = st[5] * rho;                                  // :52
    const double cr = st[4] * rho;
    const double rhobar = hypot(cr, thetanew);                            // :53
    st[4] = cr / rhobar;                                                  // :54 cbar
    st[5] = thetanew / rhobar;                                            // :55 sbar
    const double zeta = st[4] * st[6];                                    // :58
    st[6] = -st[5] * st[6];                                               // :59 zetabar
    const double c_hbar = (thetabar * rho) / (rhoold * rhobarold);        // :64
    const double c_x = zeta / (rho * rhobar);                             // :66
    const double c_h = thetanew / rho;                                    // :67
    coef[0] = (T)c_hbar;
    coef[1] = (T)c_x;
    coef[2] = (T)c_h;
    const double f = st[7];
    const double m5[5] = {1.0, 0.0, f, c_hbar, c_x}, n5[5] = {beta, alpha_k, f, c_hbar, c_x};
    for (int i = 0; i < 5; ++i) {
        cfm[i] = m5[i];
        cfn[i] = n5[i];
    }
    st[0] = alpha;
    st[2] = rho;
    st[3] = rhobar;
    st[7] = c_h;
}

// The n-space LSMR step (lsmr_solver.m:40, :61-67) with device coefficients: v = v / alpha
// (alpha = (T)sqrt(*ssa); a zero alpha leaves v, :40), hbar = h - c_hbar hbar (k = 0: h), x += c_x hbar,
// h = v - c_h h -- x, h, hbar untouched once an earlier iteration met the stop test -- and, with
// parts, the partials of ||x - x_true||^2 (:72) in k_lsqr_step's layout.
template <typename T, bool FIRST, bool VEC>
__global__ __launch_bounds__(BS) void k_lsmr_step(int64_t n, T* __restrict__ x, T* __restrict__ h,
                                                  T* __restrict__ hbar, T* __restrict__ v, const T* ssa,
                                                  const T* coef, const double* st, int k, const T* __restrict__ xt,
                                                  T* __restrict__ parts) {
    __shared__ T sh[4];
    const T alpha = (T)sqrt((double)*ssa);
    const bool live = !(st[8] != 0.0 && st[8] < (double)(k + 1));
    const T c_hbar = coef[0], c_x = coef[1], c_h = coef[2];
    T acc = 0;
    grid_elems<T, VEC>(n, [&](int64_t i, auto wc) {
        constexpr int W = decltype(wc)::value;
        T vv[W], xx[W], hh[W], hb[W], tt[W];
        vload<W>(v, i, vv);
        vload<W>(x, i, xx);
        if (live) {
            vload<W>(h, i, hh);
            if (!FIRST) vload<W>(hbar, i, hb);
        }
        if (parts) vload<W>(xt, i, tt);
#pragma unroll
        for (int e = 0; e < W; ++e) {
            if (alpha > T(0)) vv[e] = vv[e] / alpha;                 // :40
            if (live) {
                if (FIRST) hb[e] = hh[e];                            // :62
                else { const T p = c_hbar * hb[e]; hb[e] = hh[e] - p; }   // :64
                const T q = c_x * hb[e];
                xx[e] = xx[e] + q;                                   // :66
                const T r = c_h * hh[e];
                hh[e] = vv[e] - r;                                   // :67
            }
            if (parts) {
                const T d = xx[e] - tt[e];
                acc += d * d;
            }
        }
        if (alpha > T(0)) vstore<W>(v, i, vv);
        if (live) {
            vstore<W>(hbar, i, hb);
            vstore<W>(x, i, xx);
            vstore<W>(h, i, hh);
        }
    });
    if (parts) {
        const T tot = block_sum_all(acc, sh);
        if (threadIdx.x == 0) parts[blockIdx.x] = tot;
    }
}

// :76 on the device: st[8] = k + 1 at the first iteration with sqrt(||r||^2) / (||b|| + eps) < tol
__global__ void k_lsmr_stop(const double* rr, double nb, double tol, double* st, int k) {
    if (threadIdx.x != 0) return;
    const double res = sqrt(rr[0]) / (nb + 0x1p-52);   // eps
    if (st[8] == 0.0 && res < tol) st[8] = (double)(k + 1);
}

// out = in / sqrt(*ss), or in when the sum is zero (lsmr_solver.m:36: if beta > 0, u = u / beta)
template <typename T>
__global__ __launch_bounds__(BS) void k_div_sqrt_nz(int64_t n, const T* __restrict__ in, T* __restrict__ out,
                                                    const T* ss) {
    const T s = (T)sqrt((double)*ss);
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
        out[i] = s > T(0) ? in[i] / s : in[i];
}

template <typename T>
void lsmr_rot(hgm_ctx* c, const T* ssb, const T* ssa, double* st, T* coef, double* cfm, double* cfn,
              const ScalarCopy<T>& cp) {
    k_lsmr_rot<T><<<1, 64, 0, c->stream>>>(ssb, ssa, st, coef, cfm, cfn, cp);
    HGM_HIP(hipGetLastError());
}

template <typename T>
void lsmr_step(hgm_ctx* c, int64_t n, T* x, T* h, T* hbar, T* v, const T* ssa, const T* coef, const double* st,
               int k, const T* xt, T* err_out) {
    const bool fuse = xt && n > SINGLE_MAX;
    const int np = fuse ? parts_for(n) : grid_for(n);
    T* parts = fuse ? c->buf<T>("red_parts", MAX_PARTS) : nullptr;
    const bool vec = al16(x) && al16(h) && al16(hbar) && al16(v) && (!xt || al16(xt));
    if (k == 0 && vec) k_lsmr_step<T, true, true><<<np, BS, 0, c->stream>>>(n, x, h, hbar, v, ssa, coef, st, k, xt, parts);
    else if (k == 0) k_lsmr_step<T, true, false><<<np, BS, 0, c->stream>>>(n, x, h, hbar, v, ssa, coef, st, k, xt, parts);
    else if (vec) k_lsmr_step<T, false, true><<<np, BS, 0, c->stream>>>(n, x, h, hbar, v, ssa, coef, st, k, xt, parts);
    else k_lsmr_step<T, false, false><<<np, BS, 0, c->stream>>>(n, x, h, hbar, v, ssa, coef, st, k, xt, parts);
    if (fuse) k_finalize<T><<<1, BS, 0, c->stream>>>(parts, np, err_out);
    HGM_HIP(hipGetLastError());
    if (xt && !fuse) sumsq_diff<T>(c, n, x, xt, err_out);
}

void lsmr_stop(hgm_ctx* c, const double* rr, double nb, double tol, double* st, int k) {
    k_lsmr_stop<<<1, 64, 0, c->stream>>>(rr, nb, tol, st, k);
    HGM_HIP(hipGetLastError());
}

template <typename T>
void div_sqrt_nz(hgm_ctx* c, int64_t n, const T* in, T* out, const T* ss) {
    k_div_sqrt_nz<T><<<grid_for(n), BS, 0, c->stream>>>(n, in, out, ss);
    HGM_HIP(hipGetLastError());
}

// LSMR monitors from kept products.  The images of the LSMR vectors under A
// and A'A follow the same recurrences as the vectors (lsmr_solver.m:61-67), fed by the raw
// products the bidiagonalisation already forms:
//   m-space: A*h_k = A*v_k - f*A*h_{k-1};  A*hbar_k = A*h_k - e*A*hbar_{k-1};  A*x_k = A*x_{k-1} + cx*A*hbar_k
//   n-space: A'A*v_k = beta_{k+1} A'u_{k+1} + alpha_k A'u_k  (A*v_k = beta_{k+1} u_{k+1} + alpha_k u_k,
//            lsmr_solver.m:34-36), then the same three updates for A'A*h, A'A*hbar, A'A*x.
// r = b - A*x (:69) and A'r = A'b - A'A*x (:71) are then norms of kept vectors.  The images are
// accumulated in fp64 for both value types.  parts[blk] = this block's sum of the squared
// monitor vector.
// cf != NULL: the coefficients [c1, c0, f, e, cx] from the device (k_lsmr_rot) instead of the arguments.
template <typename T, bool FIRST>
__global__ __launch_bounds__(BS) void k_lsmr_mon(int64_t n, const T* __restrict__ p1, const T* __restrict__ p0,
                                                 double c1, double c0, double* __restrict__ Ih,
                                                 double* __restrict__ Ihb, double* __restrict__ Ix,
                                                 const T* __restrict__ rhs, double f, double e, double cx,
                                                 double* __restrict__ parts, const double* __restrict__ cf) {
    __shared__ double sh[4];
    if (cf) {
        c1 = cf[0];
        c0 = cf[1];
        f = cf[2];
        e = cf[3];
        cx = cf[4];
    }
    double acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
        double iv;                                          // image of v_k
        if (p0) { const double a = c1 * (double)p1[i], b = c0 * (double)p0[i]; iv = a + b; }
        else iv = (double)p1[i];
        double ih, ihb;
        if (FIRST) { ih = iv; ihb = ih; }                  // h_0 = v_0 (:25), hbar_0 = h_0 (:62)
        else {
            const double q = f * Ih[i];
            ih = iv - q;
            const double w = e * Ihb[i];
            ihb = ih - w;
        }
        const double s = cx * ihb;
        const double ix = Ix[i] + s;
        Ih[i] = ih;
        Ihb[i] = ihb;
        Ix[i] = ix;
        const double d = (double)rhs[i] - ix;
        acc += d * d;
    }
    const double tot = block_sum_all(acc, sh);
    if (threadIdx.x == 0) parts[blockIdx.x] = tot;
}

// The n-space monitor of the fp32 solves in carried-residual form: the images of h and hbar and
// the normal-equations residual Ir = A'b - A'A*x itself (Ir_0 = A'b) are stored in T and updated in
// double, Ir_k = Ir_{k-1} - cx * image(hbar_k); parts = sum Ir_k^2 (the rounded values carried on).
// Carrying Ir instead of image(x) keeps the small residual from a cancellation against A'b, so T
// storage holds its relative accuracy; it moves 3 T arrays twice plus p1, p0 per iteration instead
// of 3 double arrays twice plus p1, p0 and A'b (C5: 0.54 against 1.0 GB).
template <typename T, bool FIRST, bool VEC>
__global__ __launch_bounds__(BS) void k_lsmr_mon_r(int64_t n, const T* __restrict__ p1, const T* __restrict__ p0,
                                                   T* __restrict__ Ih, T* __restrict__ Ihb, T* __restrict__ Ir,
                                                   double* __restrict__ parts, const double* __restrict__ cf) {
    __shared__ double sh[4];
    const double c1 = cf[0], c0 = cf[1], f = cf[2], e = cf[3], cx = cf[4];
    double acc = 0;
    grid_elems<T, VEC>(n, [&](int64_t i, auto wc) {
        constexpr int W = decltype(wc)::value;
        T a[W], b[W], h[W], hb[W], r[W];
        vload<W>(p1, i, a);
        vload<W>(p0, i, b);
        if (!FIRST) {
            vload<W>(Ih, i, h);
            vload<W>(Ihb, i, hb);
        }
        vload<W>(Ir, i, r);
#pragma unroll
        for (int u = 0; u < W; ++u) {
            const double x1 = c1 * (double)a[u], x0 = c0 * (double)b[u];
            const double iv = x1 + x0;
            double ih, ihb;
            if (FIRST) { ih = iv; ihb = ih; }
            else {
                const double q = f * (double)h[u];
                ih = iv - q;
                const double w = e * (double)hb[u];
                ihb = ih - w;
            }
            const double s = cx * ihb;
            const double ir = (double)r[u] - s;
            h[u] = (T)ih;
            hb[u] = (T)ihb;
            r[u] = (T)ir;
            const double rr = (double)r[u];
            acc += rr * rr;
        }
        vstore<W>(Ih, i, h);
        vstore<W>(Ihb, i, hb);
        vstore<W>(Ir, i, r);
    });
    const double tot = block_sum_all(acc, sh);
    if (threadIdx.x == 0) parts[blockIdx.x] = tot;
}

template <typename T>
void lsmr_monitor_r(hgm_ctx* c, int64_t n, const T* p1, const T* p0, T* Ih, T* Ihb, T* Ir, bool first, double* out,
                    const double* cf) {
    const int np = parts_for(n);
    double* parts = c->buf<double>("lsmr_mon_parts", MAX_PARTS);
    const bool vec = al16(p1) && al16(p0) && al16(Ih) && al16(Ihb) && al16(Ir);
#define HGM_MONR(F, V) k_lsmr_mon_r<T, F, V><<<np, BS, 0, c->stream>>>(n, p1, p0, Ih, Ihb, Ir, parts, cf)
    if (first && vec) HGM_MONR(true, true);
    else if (first) HGM_MONR(true, false);
    else if (vec) HGM_MONR(false, true);
    else HGM_MONR(false, false);
#undef HGM_MONR
    k_finalize<double><<<1, BS, 0, c->stream>>>(parts, np, out);
    HGM_HIP(hipGetLastError());
}

// k_lsmr_step and k_lsmr_mon_r in one pass over the n-space (the fp32 one-pass LSMR with x_true):
// the two kernels walk the same elements in the same grid (parts_for(n) blocks, grid_elems) and
// touch disjoint vectors, so each of the two block sums -- and every element -- has the bits of
// the two separate launches; one launch boundary and one sweep of the grid instead of two.
template <typename T, bool FIRST>
__global__ __launch_bounds__(BS) void k_lsmr_step_mon(int64_t n, T* __restrict__ x, T* __restrict__ h,
                                                      T* __restrict__ hbar, T* __restrict__ v, const T* ssa,
                                                      const T* coef, const double* st, int k, const T* __restrict__ xt,
                                                      T* __restrict__ parts_e, const T* __restrict__ p1,
                                                      const T* __restrict__ p0, T* __restrict__ Ih, T* __restrict__ Ihb,
                                                      T* __restrict__ Ir, double* __restrict__ parts_m,
                                                      const double* __restrict__ cf) {
    __shared__ T sh[4];
    __shared__ double shm[4];
    const T alpha = (T)sqrt((double)*ssa);
    const bool live = !(st[8] != 0.0 && st[8] < (double)(k + 1));
    const T c_hbar = coef[0], c_x = coef[1], c_h = coef[2];
    const double c1 = cf[0], c0 = cf[1], f = cf[2], e = cf[3], cx = cf[4];
    T acc = 0;
    double accm = 0;
    grid_elems<T, true>(n, [&](int64_t i, auto wc) {
        constexpr int W = decltype(wc)::value;
        {   // k_lsmr_step's element body
            T vv[W], xx[W], hh[W], hb[W], tt[W];
            vload<W>(v, i, vv);
            vload<W>(x, i, xx);
            if (live) {
                vload<W>(h, i, hh);
                if (!FIRST) vload<W>(hbar, i, hb);
            }
            vload<W>(xt, i, tt);
#pragma unroll
            for (int u = 0; u < W; ++u) {
                if (alpha > T(0)) vv[u] = vv[u] / alpha;
                if (live) {
                    if (FIRST) hb[u] = hh[u];
                    else { const T p = c_hbar * hb[u]; hb[u] = hh[u] - p; }
                    const T q = c_x * hb[u];
                    xx[u] = xx[u] + q;
                    const T r = c_h * hh[u];
                    hh[u] = vv[u] - r;
                }
                const T d = xx[u] - tt[u];
                acc += d * d;
            }
            if (alpha > T(0)) vstore<W>(v, i, vv);
            if (live) {
                vstore<W>(hbar, i, hb);
                vstore<W>(x, i, xx);
                vstore<W>(h, i, hh);
            }
        }
        {   // k_lsmr_mon_r's element body
            T a[W], b[W], hm[W], hbm[W], r[W];
            vload<W>(p1, i, a);
            vload<W>(p0, i, b);
            if (!FIRST) {
                vload<W>(Ih, i, hm);
                vload<W>(Ihb, i, hbm);
            }
            vload<W>(Ir, i, r);
#pragma unroll
            for (int u = 0; u < W; ++u) {
                const double x1 = c1 * (double)a[u], x0 = c0 * (double)b[u];
                const double iv = x1 + x0;
                double ih, ihb;
                if (FIRST) { ih = iv; ihb = ih; }
                else {
                    const double q = f * (double)hm[u];
                    ih = iv - q;
                    const double w = e * (double)hbm[u];
                    ihb = ih - w;
                }
                const double s_ = cx * ihb;
                const double ir = (double)r[u] - s_;
                hm[u] = (T)ih;
                hbm[u] = (T)ihb;
                r[u] = (T)ir;
                const double rr = (double)r[u];
                accm += rr * rr;
            }
            vstore<W>(Ih, i, hm);
            vstore<W>(Ihb, i, hbm);
            vstore<W>(Ir, i, r);
        }
    });
    const T tot = block_sum_all(acc, sh);
    const double totm = block_sum_all(accm, shm);
    if (threadIdx.x == 0) {
        parts_e[blockIdx.x] = tot;
        parts_m[blockIdx.x] = totm;
    }
}

// The fused pair when it gives the separate launches' bits (x_true given, the partial-sum grid,
// 16-byte aligned vectors); false: the caller runs lsmr_step and lsmr_monitor_r.
template <typename T>
bool lsmr_step_mon(hgm_ctx* c, int64_t n, T* x, T* h, T* hbar, T* v, const T* ssa, const T* coef, const double* st,
                   int k, const T* xt, T* err_out, const T* p1, const T* p0, T* Ih, T* Ihb, T* Ir, bool first,
                   double* mon_out, const double* cf) {
    if (!c->num.lsmr_fuse_nmon || !xt || n <= SINGLE_MAX) return false;
    if (!(al16(x) && al16(h) && al16(hbar) && al16(v) && al16(xt) && al16(p1) && al16(p0) && al16(Ih) && al16(Ihb) &&
          al16(Ir)))
        return false;
    const int np = parts_for(n);
    T* parts_e = c->buf<T>("red_parts", MAX_PARTS);
    double* parts_m = c->buf<double>("lsmr_mon_parts", MAX_PARTS);
    if (first)
        k_lsmr_step_mon<T, true><<<np, BS, 0, c->stream>>>(n, x, h, hbar, v, ssa, coef, st, k, xt, parts_e, p1, p0, Ih,
                                                           Ihb, Ir, parts_m, cf);
    else
        k_lsmr_step_mon<T, false><<<np, BS, 0, c->stream>>>(n, x, h, hbar, v, ssa, coef, st, k, xt, parts_e, p1, p0, Ih,
                                                            Ihb, Ir, parts_m, cf);
    k_finalize<T><<<1, BS, 0, c->stream>>>(parts_e, np, err_out);
    k_finalize<double><<<1, BS, 0, c->stream>>>(parts_m, np, mon_out);
    HGM_HIP(hipGetLastError());
    return true;
}

template <typename T>
void lsmr_monitor(hgm_ctx* c, int64_t n, const T* p1, const T* p0, double c1, double c0, double* Ih, double* Ihb,
                  double* Ix, const T* rhs, double f, double e, double cx, bool first, double* out, const double* cf) {
    const int np = parts_for(n);
    double* parts = c->buf<double>("lsmr_mon_parts", MAX_PARTS);
    if (first)
        k_lsmr_mon<T, true><<<np, BS, 0, c->stream>>>(n, p1, p0, c1, c0, Ih, Ihb, Ix, rhs, f, e, cx, parts, cf);
    else
        k_lsmr_mon<T, false><<<np, BS, 0, c->stream>>>(n, p1, p0, c1, c0, Ih, Ihb, Ix, rhs, f, e, cx, parts, cf);
    k_finalize<double><<<1, BS, 0, c->stream>>>(parts, np, out);
    HGM_HIP(hipGetLastError());
}

// out = a * in
template <typename T>
__global__ __launch_bounds__(BS) void k_scale(int64_t n, const T* __restrict__ in, T* __restrict__ out, T a) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) out[i] = a * in[i];
}
template <typename T> void scale(hgm_ctx* c, int64_t n, const T* in, T* out, T a) {
    k_scale<T><<<grid_for(n), BS, 0, c->stream>>>(n, in, out, a);
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

// Deterministic pseudo-random vector in (-1, 1): x_i = splitmix64(seed + i) scaled (the start
// vector of the Ritz Arnoldi in bounds.cpp; the same bits on every device and run).
template <typename T>
__global__ __launch_bounds__(BS) void k_fill_hash(int64_t n, T* x, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
        uint64_t z = seed + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        x[i] = (T)((double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0);
    }
}
template <typename T> void fill_hash(hgm_ctx* c, int64_t n, T* x, uint64_t seed) {
    k_fill_hash<T><<<grid_for(n), BS, 0, c->stream>>>(n, x, seed);
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
    template void recon<T>(hgm_ctx*, int64_t, int, const T*, int64_t, const T*, T*, const T*, T*, int64_t, \
                           const T*, int64_t, const T*, T*);                                   \
    template void normalize_to<T>(hgm_ctx*, int64_t, T*, T*);                                                        \
    template void mgs<T>(hgm_ctx*, int64_t, T*, int64_t, int, T*, bool, const T*, const MdotJob<T>*, PendNorm<T>*,   \
                         const T*, const T*, T*, const double*, double*);                      \
    template void cgs2<T>(hgm_ctx*, int64_t, T*, int64_t, int, T*, bool);                      \
    template void gemv<T>(hgm_ctx*, int64_t, int, const T*, int64_t, const T*, T*, int);       \
    template void div_scalar<T>(hgm_ctx*, int64_t, const T*, T*, T);                           \
    template void lsqr_update<T>(hgm_ctx*, int64_t, T*, T*, const T*, T, T);                   \
    template void lsqr_rot<T>(hgm_ctx*, const T*, const T*, double*, T*, double*, int, double, double,   \
                              const ScalarCopy<T>&);                                            \
    template void lsqr_step<T>(hgm_ctx*, int64_t, T*, T*, T*, const T*, const T*, const double*, int, const T*, T*); \
    template void div_sqrt<T>(hgm_ctx*, int64_t, const T*, T*, const T*);                     \
    template void lsmr_update<T>(hgm_ctx*, int64_t, T*, T*, T*, const T*, T, T, T, bool);      \
    template void lsmr_monitor<T>(hgm_ctx*, int64_t, const T*, const T*, double, double, double*, double*, \
                                  double*, const T*, double, double, double, bool, double*, const double*); \
    template void lsmr_rot<T>(hgm_ctx*, const T*, const T*, double*, T*, double*, double*,         \
                              const ScalarCopy<T>&);                                            \
    template void lsmr_monitor_r<T>(hgm_ctx*, int64_t, const T*, const T*, T*, T*, T*, bool, double*, \
                                    const double*);                                            \
    template void lsmr_step<T>(hgm_ctx*, int64_t, T*, T*, T*, T*, const T*, const T*, const double*, int, \
                               const T*, T*);                                                  \
    template bool lsmr_step_mon<T>(hgm_ctx*, int64_t, T*, T*, T*, T*, const T*, const T*, const double*, int, \
                                   const T*, T*, const T*, const T*, T*, T*, T*, bool, double*, const double*); \
    template void div_sqrt_nz<T>(hgm_ctx*, int64_t, const T*, T*, const T*);                  \
    template void fill<T>(hgm_ctx*, int64_t, T*, T);                                           \
    template void scale<T>(hgm_ctx*, int64_t, const T*, T*, T);                                \
    template void fill_hash<T>(hgm_ctx*, int64_t, T*, uint64_t);                               \
    template void convert<T>(hgm_ctx*, int64_t, const double*, T*);                            \
    template void convert_back<T>(hgm_ctx*, int64_t, const T*, double*);                       \
    template void fro2<T>(hgm_ctx*, const hgm_mat*, double*);                                   \
    template void fixed_reduce<T>(hgm_ctx*, int, int64_t, const T*, const T*, int64_t, const T*, const T*, T*);

HGM_INST(double)
HGM_INST(float)

}  // namespace hgm
