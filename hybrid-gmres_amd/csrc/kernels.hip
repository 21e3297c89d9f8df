// HIP kernels of the Arnoldi/GMRES + Golub-Kahan inner loop, written for gfx950 (CDNA4).
//
// Design:
//  * SpMV: CSR, one G-lane group per row (G = 64 -> one wave per row for the long
//    ray-major rows of A; G = 8..32 for the short pixel-major rows of B / A^T), loads
//    of val/col coalesced inside a group, products summed per lane then reduced with a
//    fixed xor-butterfly (deterministic, no atomics).  Epilogues of the reference's
//    operator closures are fused into the store: `B*(A*v) + lambda*v`
//    (hybrid_*_rtp.m:6), `A*v - alpha*u` (lsqr_solver.m:22), `A'*u - beta*v`
//    (lsqr_solver.m:26) and `b - A*x` (hybrid_*_rtp.m:32/35), each with MATLAB's two
//    roundings (the file is compiled with -ffp-contract=off).
//  * MGS (hybrid_*_rtp.m:20-26): one launch per Gram-Schmidt pass j fusing
//    axpy_j (v -= h_j q_j) with the inner product of the NEXT column (q_{j+1}' v).  The
//    grid-wide sum of pass j's block partials is re-reduced, in a fixed order, by
//    every block of pass j+1 (identical bits in every block), so no separate reduce
//    launch and no host round trip is needed between passes.
//  * All reductions: per-lane sums -> wave butterfly -> 4-wave LDS sum in fixed order.
#include "internal.h"

namespace hgm {

template <typename T> struct V2;
template <> struct V2<double> { using t = double2; };
template <> struct V2<float> { using t = float2; };

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Block (256 threads) sum, result broadcast to every thread.  Fixed order.
template <typename T>
__device__ __forceinline__ T block_sum_all(T v, T* sh) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    T r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
    __syncthreads();
    return r;
}

// Sum of np partials (np <= MAX_PARTS) — same bits in every block that calls it.
template <typename T>
__device__ __forceinline__ T reduce_parts(const T* __restrict__ p, int np, T* sh) {
    T a = 0;
    for (int i = threadIdx.x; i < np; i += BS) a += p[i];
    return block_sum_all(a, sh);
}

int parts_for(int64_t n) {
    // >= 2 element pairs per thread, up to MAX_PARTS blocks (256 CUs x 4)
    int64_t nb = (n + 2 * BS * 2 - 1) / (2 * BS * 2);
    if (nb < 1) nb = 1;
    if (nb > MAX_PARTS) nb = MAX_PARTS;
    return (int)nb;
}

// ------------------------------------------------------------------------------
// SpMV
// ------------------------------------------------------------------------------
template <typename T, int EPI>
__device__ __forceinline__ T apply_epi(T t, T a, const T* __restrict__ z, int64_t i) {
    if (EPI == EPI_ADD) { T s = a * z[i]; return t + s; }
    if (EPI == EPI_SUB) { T s = a * z[i]; return t - s; }
    if (EPI == EPI_RSUB) return z[i] - t;
    return t;
}

template <bool NT, typename V>
__device__ __forceinline__ V ld(const V* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// native clang vectors (the nontemporal builtin does not take HIP_vector_type)
typedef double nd2 __attribute__((ext_vector_type(2)));
typedef float nf2 __attribute__((ext_vector_type(2)));
typedef int ni2 __attribute__((ext_vector_type(2)));
template <typename T> struct NV2;
template <> struct NV2<double> { using t = nd2; };
template <> struct NV2<float> { using t = nf2; };

// XCD-aware block order (speed only, never correctness): consecutive logical row blocks
// run on the same XCD so neighbouring rays share x lines in that XCD's L2
// (cdna_hip_programming.md §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
    const int64_t q = nb / 8, r = nb % 8, xcd = b % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// One G-lane group per CSR row.  VEC: each lane streams pairs of entries with 16-byte
// value loads and 8-byte index loads (row heads/tails peeled to keep them aligned).
// NT: nontemporal (streaming) loads for val/col so they do not evict x from L2/MALL.
// Per-lane partial of the dot product of entries [s, e) with x, lane gl of a G-lane group.
template <typename T, int G, bool VEC, bool NT>
__device__ __forceinline__ T seg_partial(int64_t s, int64_t e, int gl, const int32_t* __restrict__ ci,
                                         const T* __restrict__ val, const T* __restrict__ x) {
    T a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    {
        if (!VEC) {
            int64_t i = s + gl;
            for (; i + 3 * G < e; i += 4 * G) {
                const int32_t c0 = ld<NT>(ci + i), c1 = ld<NT>(ci + i + G), c2 = ld<NT>(ci + i + 2 * G),
                              c3 = ld<NT>(ci + i + 3 * G);
                const T v0 = ld<NT>(val + i), v1 = ld<NT>(val + i + G), v2 = ld<NT>(val + i + 2 * G),
                        v3 = ld<NT>(val + i + 3 * G);
                a0 += v0 * x[c0];
                a1 += v1 * x[c1];
                a2 += v2 * x[c2];
                a3 += v3 * x[c3];
            }
            for (; i < e; i += G) a0 += ld<NT>(val + i) * x[ld<NT>(ci + i)];
        } else {
            using T2 = typename NV2<T>::t;
            using I2 = ni2;
            const int64_t s2 = (s + 1) & ~int64_t(1);     // first even index >= s
            const int64_t e2 = e & ~int64_t(1);           // last even bound <= e
            if (gl == 0 && s < s2 && s < e) a0 += ld<NT>(val + s) * x[ld<NT>(ci + s)];
            if (gl == G - 1 && e2 < e && e2 >= s2) a1 += ld<NT>(val + e2) * x[ld<NT>(ci + e2)];
            int64_t i = s2 + 2 * gl;
            for (; i + 2 * G < e2; i += 4 * G) {
                const I2 c0 = ld<NT>(reinterpret_cast<const I2*>(ci + i));
                const I2 c1 = ld<NT>(reinterpret_cast<const I2*>(ci + i + 2 * G));
                const T2 v0 = ld<NT>(reinterpret_cast<const T2*>(val + i));
                const T2 v1 = ld<NT>(reinterpret_cast<const T2*>(val + i + 2 * G));
                a0 += v0.x * x[c0.x];
                a1 += v0.y * x[c0.y];
                a2 += v1.x * x[c1.x];
                a3 += v1.y * x[c1.y];
            }
            for (; i < e2; i += 2 * G) {
                const I2 c0 = ld<NT>(reinterpret_cast<const I2*>(ci + i));
                const T2 v0 = ld<NT>(reinterpret_cast<const T2*>(val + i));
                a0 += v0.x * x[c0.x];
                a1 += v0.y * x[c0.y];
            }
        }
    }
    return (a0 + a1) + (a2 + a3);
}

template <typename T, int G>
__device__ __forceinline__ T group_sum(T acc) {
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    return acc;
}

template <typename T, int G, int EPI, bool VEC, bool NT>
__global__ __launch_bounds__(BS) void k_spmv(int64_t rows, const int64_t* __restrict__ rp,
                                             const int32_t* __restrict__ ci,
                                             const T* __restrict__ val, const T* __restrict__ x,
                                             T* __restrict__ y, T a, const T* __restrict__ z, int xcd) {
    constexpr int RPB = BS / G;
    const int64_t blk = xcd ? xcd_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int64_t row = blk * RPB + threadIdx.x / G;
    const int gl = threadIdx.x & (G - 1);
    T acc = 0;
    if (row < rows) acc = seg_partial<T, G, VEC, NT>(rp[row], rp[row + 1], gl, ci, val, x);
    acc = group_sum<T, G>(acc);
    if (gl == 0 && row < rows) y[row] = apply_epi<T, EPI>(acc, a, z, row);
}

// Column-banded SpMV: work items (band b, block of RPB rows) in band-major order, grid-
// stride, so the blocks resident at any moment gather x from one band's slice (L2-
// resident).  Writes the per-band partial ypart[b*rows + r]; k_band_reduce sums them.
template <typename T, int G, bool VEC, bool NT>
__global__ __launch_bounds__(BS) void k_spmv_band(int64_t rows, int nbands, const int64_t* __restrict__ brp,
                                                  const int32_t* __restrict__ ci, const T* __restrict__ val,
                                                  const T* __restrict__ x, T* __restrict__ ypart) {
    constexpr int RPB = BS / G;
    const int64_t rb_per_band = (rows + RPB - 1) / RPB;
    const int64_t items = rb_per_band * nbands;
    const int gl = threadIdx.x & (G - 1);
    for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const int64_t b = it / rb_per_band;
        const int64_t row = (it - b * rb_per_band) * RPB + threadIdx.x / G;
        T acc = 0;
        if (row < rows) {
            const int64_t* p = brp + b * rows + row;
            acc = seg_partial<T, G, VEC, NT>(p[0], p[1], gl, ci, val, x);
        }
        acc = group_sum<T, G>(acc);
        if (gl == 0 && row < rows) ypart[b * rows + row] = acc;
    }
}

// ------------------------------------------------------------------------------
// nnz-balanced streaming SpMV over segments (rows, or (band,row) pairs).
// Block k owns entries [k*CH, (k+1)*CH): it streams them with 16-byte loads, stages the
// products in LDS, then G-lane groups reduce every segment that STARTS in the chunk
// (fo[k] .. fo[k+1]) plus the head part of the segment that started earlier.  Complete
// segments are written (with the epilogue); a segment running past the chunk leaves its
// partial in tail[k] and every later chunk's share in head[j]; k_stream_fixup adds them
// in chunk order.  Fixed chunking => fixed summation order => bitwise reproducible.
// ------------------------------------------------------------------------------
template <typename T, int G, int EPI, bool NT>
__global__ __launch_bounds__(BS) void k_spmv_stream(int64_t nnz, int64_t nseg, const int64_t* __restrict__ sp,
                                                    const int32_t* __restrict__ fo, const int32_t* __restrict__ ci,
                                                    const T* __restrict__ val, const T* __restrict__ x,
                                                    T* __restrict__ out, T a, const T* __restrict__ z,
                                                    T* __restrict__ head, T* __restrict__ tail) {
    using T2 = typename NV2<T>::t;
    __shared__ T prod[SCH];
    const int64_t k = blockIdx.x;
    const int64_t c0 = k * SCH;
    const int64_t c1 = (c0 + SCH < nnz) ? c0 + SCH : nnz;
    const int n = (int)(c1 - c0);
    if (n == SCH) {
#pragma unroll
        for (int u = 0; u < SCH / (2 * BS); ++u) {
            const int j = 2 * threadIdx.x + u * 2 * BS;
            const T2 v = ld<NT>(reinterpret_cast<const T2*>(val + c0 + j));
            const ni2 cc = ld<NT>(reinterpret_cast<const ni2*>(ci + c0 + j));
            prod[j] = v.x * x[cc.x];
            prod[j + 1] = v.y * x[cc.y];
        }
    } else {
        for (int j = threadIdx.x; j < n; j += BS) prod[j] = val[c0 + j] * x[ci[c0 + j]];
    }
    __syncthreads();
    const int64_t s_begin = fo[k], s_end = fo[k + 1];
    const int has_head = (s_begin > 0 && sp[s_begin] > c0) ? 1 : 0;
    const int64_t ntasks = (s_end - s_begin) + has_head;
    const int gid = threadIdx.x / G, gl = threadIdx.x & (G - 1);
    constexpr int NG = BS / G;
    for (int64_t t = gid; t < ntasks; t += NG) {
        int64_t s, lo, hi;
        if (has_head && t == 0) {
            s = s_begin - 1;
            lo = c0;
        } else {
            s = s_begin + t - has_head;
            lo = sp[s];
        }
        const int64_t send = sp[s + 1];
        hi = send < c1 ? send : c1;
        T acc = 0;
        for (int64_t i = lo + gl; i < hi; i += G) acc += prod[i - c0];
        acc = group_sum<T, G>(acc);
        if (gl == 0) {
            if (has_head && t == 0) head[k] = acc;
            else if (send > c1) tail[k] = acc;
            else out[s] = apply_epi<T, EPI>(acc, a, z, s);
        }
    }
}

template <typename T, int EPI>
__global__ __launch_bounds__(BS) void k_stream_fixup(int64_t nnz, int64_t nchunks, const int64_t* __restrict__ sp,
                                                     const int32_t* __restrict__ fo, T* __restrict__ out, T a,
                                                     const T* __restrict__ z, const T* __restrict__ head,
                                                     const T* __restrict__ tail) {
    for (int64_t k = (int64_t)blockIdx.x * BS + threadIdx.x; k < nchunks; k += (int64_t)gridDim.x * BS) {
        const int64_t s_begin = fo[k], s_end = fo[k + 1];
        if (s_end <= s_begin) continue;
        const int64_t s = s_end - 1;
        const int64_t c1 = (k + 1) * SCH < nnz ? (k + 1) * SCH : nnz;
        if (sp[s + 1] <= c1) continue;
        T sum = tail[k];
        for (int64_t j = k + 1; j < nchunks; ++j) {
            sum += head[j];
            const int64_t cj1 = (j + 1) * SCH < nnz ? (j + 1) * SCH : nnz;
            if (sp[s + 1] <= cj1) break;
        }
        out[s] = apply_epi<T, EPI>(sum, a, z, s);
    }
}

template <typename T, int EPI>
__global__ __launch_bounds__(BS) void k_fill_epi(int64_t n, T* __restrict__ out, T a, const T* __restrict__ z) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
        out[i] = apply_epi<T, EPI>(T(0), a, z, i);
}

template <typename T, int G, int EPI, bool NT>
static void launch_stream_e(hipStream_t st, const SegIndex& si, const int32_t* ci, const T* val, const T* x, T* out,
                            T a, const T* z, T* head, T* tail) {
    if (si.nnz == 0) {
        int64_t g = (si.nseg + BS - 1) / BS;
        if (g > 4096) g = 4096;
        if (g > 0) k_fill_epi<T, EPI><<<g, BS, 0, st>>>(si.nseg, out, a, z);
        return;
    }
    k_spmv_stream<T, G, EPI, NT><<<si.nchunks, BS, 0, st>>>(si.nnz, si.nseg, si.sp, si.fo, ci, val, x, out, a, z,
                                                             head, tail);
    int64_t g = (si.nchunks + BS - 1) / BS;
    if (g > 4096) g = 4096;
    k_stream_fixup<T, EPI><<<g, BS, 0, st>>>(si.nnz, si.nchunks, si.sp, si.fo, out, a, z, head, tail);
}

template <typename T, int G, bool NT>
static void launch_stream_g(hipStream_t st, const SegIndex& si, const int32_t* ci, const T* val, const T* x, T* out,
                            int epi, T a, const T* z, T* head, T* tail) {
    switch (epi) {
        case EPI_NONE: launch_stream_e<T, G, EPI_NONE, NT>(st, si, ci, val, x, out, a, z, head, tail); break;
        case EPI_ADD: launch_stream_e<T, G, EPI_ADD, NT>(st, si, ci, val, x, out, a, z, head, tail); break;
        case EPI_SUB: launch_stream_e<T, G, EPI_SUB, NT>(st, si, ci, val, x, out, a, z, head, tail); break;
        default: launch_stream_e<T, G, EPI_RSUB, NT>(st, si, ci, val, x, out, a, z, head, tail); break;
    }
}

template <typename T>
static void spmv_stream(hgm_ctx* c, const SegIndex& si, int G, bool nt, const int32_t* ci, const T* val, const T* x,
                        T* out, int epi, T a, const T* z) {
    T* head = c->buf<T>("stream_head", si.nchunks + 1);
    T* tail = c->buf<T>("stream_tail", si.nchunks + 1);
    hipStream_t st = c->stream;
#define HGM_SG(GG)                                                                              \
    if (nt) launch_stream_g<T, GG, true>(st, si, ci, val, x, out, epi, a, z, head, tail);      \
    else launch_stream_g<T, GG, false>(st, si, ci, val, x, out, epi, a, z, head, tail);
    switch (G) {
        case 64: HGM_SG(64) break;
        case 32: HGM_SG(32) break;
        case 16: HGM_SG(16) break;
        case 8: HGM_SG(8) break;
        default: HGM_SG(4) break;
    }
#undef HGM_SG
}

// y[r] = epi( sum_b ypart[b*rows + r] ), bands summed in increasing b (deterministic)
template <typename T, int EPI>
__global__ __launch_bounds__(BS) void k_band_reduce(int64_t rows, int nbands, const T* __restrict__ ypart,
                                                    T* __restrict__ y, T a, const T* __restrict__ z) {
    for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < rows; r += (int64_t)gridDim.x * BS) {
        T s = 0;
        for (int b = 0; b < nbands; ++b) s += ypart[(int64_t)b * rows + r];
        y[r] = apply_epi<T, EPI>(s, a, z, r);
    }
}

int pick_group(int64_t rows, int64_t nnz) {
    const double avg = rows > 0 ? (double)nnz / (double)rows : 0.0;
    if (avg >= 128) return 64;
    if (avg >= 40) return 32;
    if (avg >= 16) return 16;
    if (avg >= 6) return 8;
    return 4;
}

template <typename T, int G, bool VEC, bool NT>
static void launch_spmv_v(hipStream_t st, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z) {
    const int64_t nb = (M->rows + (BS / G) - 1) / (BS / G);
    if (nb == 0) return;
    const T* val = reinterpret_cast<const T*>(M->val);
    const int xcd = (M->variant & SPMV_XCD) ? 1 : 0;
    switch (epi) {
        case EPI_NONE: k_spmv<T, G, EPI_NONE, VEC, NT><<<nb, BS, 0, st>>>(M->rows, M->rp, M->ci, val, x, y, a, z, xcd); break;
        case EPI_ADD: k_spmv<T, G, EPI_ADD, VEC, NT><<<nb, BS, 0, st>>>(M->rows, M->rp, M->ci, val, x, y, a, z, xcd); break;
        case EPI_SUB: k_spmv<T, G, EPI_SUB, VEC, NT><<<nb, BS, 0, st>>>(M->rows, M->rp, M->ci, val, x, y, a, z, xcd); break;
        default: k_spmv<T, G, EPI_RSUB, VEC, NT><<<nb, BS, 0, st>>>(M->rows, M->rp, M->ci, val, x, y, a, z, xcd); break;
    }
}

template <typename T, int G>
static void launch_spmv_g(hipStream_t st, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z) {
    const bool vec = M->variant & SPMV_VEC, nt = M->variant & SPMV_NT;
    if (vec && nt) launch_spmv_v<T, G, true, true>(st, M, x, y, epi, a, z);
    else if (vec) launch_spmv_v<T, G, true, false>(st, M, x, y, epi, a, z);
    else if (nt) launch_spmv_v<T, G, false, true>(st, M, x, y, epi, a, z);
    else launch_spmv_v<T, G, false, false>(st, M, x, y, epi, a, z);
}

template <typename T, int G, bool VEC, bool NT>
static void launch_band_v(hipStream_t st, const hgm_mat* M, const T* x, T* yp) {
    constexpr int RPB = BS / G;
    const int64_t items = (M->rows + RPB - 1) / RPB * M->nbands;
    int64_t grid = 256 * 8;                      // ~all resident blocks, grid-stride in band-major order
    if (grid > items) grid = items;
    if (grid < 1) return;
    k_spmv_band<T, G, VEC, NT><<<grid, BS, 0, st>>>(M->rows, M->nbands, M->brp, M->bci,
                                                    reinterpret_cast<const T*>(M->bval), x, yp);
}

template <typename T, int G>
static void launch_band_g(hipStream_t st, const hgm_mat* M, const T* x, T* yp) {
    const bool vec = M->variant & SPMV_VEC, nt = M->variant & SPMV_NT;
    if (vec && nt) launch_band_v<T, G, true, true>(st, M, x, yp);
    else if (vec) launch_band_v<T, G, true, false>(st, M, x, yp);
    else if (nt) launch_band_v<T, G, false, true>(st, M, x, yp);
    else launch_band_v<T, G, false, false>(st, M, x, yp);
}

template <typename T>
static void spmv_banded(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z) {
    T* yp = c->buf<T>("band_part", (size_t)M->nbands * M->rows + 1);
    switch (M->bgroup) {
        case 64: launch_band_g<T, 64>(c->stream, M, x, yp); break;
        case 32: launch_band_g<T, 32>(c->stream, M, x, yp); break;
        case 16: launch_band_g<T, 16>(c->stream, M, x, yp); break;
        case 8: launch_band_g<T, 8>(c->stream, M, x, yp); break;
        default: launch_band_g<T, 4>(c->stream, M, x, yp); break;
    }
    int64_t g = (M->rows + BS - 1) / BS;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    switch (epi) {
        case EPI_NONE: k_band_reduce<T, EPI_NONE><<<g, BS, 0, c->stream>>>(M->rows, M->nbands, yp, y, a, z); break;
        case EPI_ADD: k_band_reduce<T, EPI_ADD><<<g, BS, 0, c->stream>>>(M->rows, M->nbands, yp, y, a, z); break;
        case EPI_SUB: k_band_reduce<T, EPI_SUB><<<g, BS, 0, c->stream>>>(M->rows, M->nbands, yp, y, a, z); break;
        default: k_band_reduce<T, EPI_RSUB><<<g, BS, 0, c->stream>>>(M->rows, M->nbands, yp, y, a, z); break;
    }
}

template <typename T, int EPI>
static void launch_band_reduce(hgm_ctx* c, const hgm_mat* M, const T* yp, T* y, T a, const T* z) {
    int64_t g = (M->rows + BS - 1) / BS;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    k_band_reduce<T, EPI><<<g, BS, 0, c->stream>>>(M->rows, M->nbands, yp, y, a, z);
}

template <typename T>
static void spmv_streamed(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z) {
    const bool nt = M->variant & SPMV_NT;
    if (M->nbands > 1) {
        T* yp = c->buf<T>("band_part", (size_t)M->nbands * M->rows + 1);
        SegIndex si{M->nnz, (int64_t)M->nbands * M->rows, stream_chunks(M->nnz), M->brp, M->bcfo};
        spmv_stream<T>(c, si, M->bsgroup, nt, M->bci, reinterpret_cast<const T*>(M->bval), x, yp, EPI_NONE, T(0),
                       nullptr);
        switch (epi) {
            case EPI_NONE: launch_band_reduce<T, EPI_NONE>(c, M, yp, y, a, z); break;
            case EPI_ADD: launch_band_reduce<T, EPI_ADD>(c, M, yp, y, a, z); break;
            case EPI_SUB: launch_band_reduce<T, EPI_SUB>(c, M, yp, y, a, z); break;
            default: launch_band_reduce<T, EPI_RSUB>(c, M, yp, y, a, z); break;
        }
    } else {
        SegIndex si{M->nnz, M->rows, stream_chunks(M->nnz), M->rp, M->cfo};
        spmv_stream<T>(c, si, M->sgroup, nt, M->ci, reinterpret_cast<const T*>(M->val), x, y, epi, a, z);
    }
}

template <typename T>
void spmv(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z, int kclass) {
    hipEvent_t t0 = nullptr;
    timing_begin(c, kclass, &t0);
    if ((M->variant & SPMV_STREAM) && (M->nbands > 1 ? M->bcfo != nullptr : M->cfo != nullptr)) {
        spmv_streamed<T>(c, M, x, y, epi, a, z);
        HGM_HIP(hipGetLastError());
        const double s = sizeof(T);
        double bytes = (double)M->nnz * (s + 4) + 8.0 * (M->rows + 1) + s * M->cols + s * M->rows;
        if (epi != EPI_NONE) bytes += s * M->rows;
        timing_end(c, kclass, t0, bytes);
        return;
    }
    if (M->nbands > 1) {
        spmv_banded<T>(c, M, x, y, epi, a, z);
        HGM_HIP(hipGetLastError());
        const double s = sizeof(T);
        double bytes = (double)M->nnz * (s + 4) + 8.0 * (M->rows + 1) + s * M->cols + s * M->rows;
        if (epi != EPI_NONE) bytes += s * M->rows;
        timing_end(c, kclass, t0, bytes);
        return;
    }
    switch (M->group) {
        case 64: launch_spmv_g<T, 64>(c->stream, M, x, y, epi, a, z); break;
        case 32: launch_spmv_g<T, 32>(c->stream, M, x, y, epi, a, z); break;
        case 16: launch_spmv_g<T, 16>(c->stream, M, x, y, epi, a, z); break;
        case 8: launch_spmv_g<T, 8>(c->stream, M, x, y, epi, a, z); break;
        default: launch_spmv_g<T, 4>(c->stream, M, x, y, epi, a, z); break;
    }
    HGM_HIP(hipGetLastError());
    // algorithmic bytes: nnz*(s+4) + 8(rows+1) + s*cols + s*rows (+ s*rows epilogue operand)
    const double s = sizeof(T);
    double bytes = (double)M->nnz * (s + 4) + 8.0 * (M->rows + 1) + s * M->cols + s * M->rows;
    if (epi != EPI_NONE) bytes += s * M->rows;
    timing_end(c, kclass, t0, bytes);
}

template <typename T, int EPI>
__global__ __launch_bounds__(BS) void k_epi(int64_t n, T* __restrict__ y, T a, const T* __restrict__ z) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
        y[i] = apply_epi<T, EPI>(y[i], a, z, i);
}

static int grid_for(int64_t n) {
    int64_t nb = (n + BS - 1) / BS;
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    return (int)nb;
}

template <typename T>
void epilogue(hgm_ctx* c, int64_t n, T* y, int epi, T a, const T* z) {
    const int g = grid_for(n);
    switch (epi) {
        case EPI_ADD: k_epi<T, EPI_ADD><<<g, BS, 0, c->stream>>>(n, y, a, z); break;
        case EPI_SUB: k_epi<T, EPI_SUB><<<g, BS, 0, c->stream>>>(n, y, a, z); break;
        case EPI_RSUB: k_epi<T, EPI_RSUB><<<g, BS, 0, c->stream>>>(n, y, a, z); break;
        default: return;
    }
    HGM_HIP(hipGetLastError());
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
    template void spmv<T>(hgm_ctx*, const hgm_mat*, const T*, T*, int, T, const T*, int);      \
    template void epilogue<T>(hgm_ctx*, int64_t, T*, int, T, const T*);                        \
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
